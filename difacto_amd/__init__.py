"""difacto_amd — DiFacto's data-parallel hot path (FM/LR forward-backward, FTRL/AdaGrad
sparse update, Localizer, device KV store) on AMD MI355X (gfx950).

The product is libdifacto_amd.so (HIP kernels behind the C-ABI in include/difacto_amd.h);
``difacto_amd.hotpath`` is its Python mirror of the reference's Loss/Updater/Store
interfaces.  Importing the package does not touch the GPU; import ``hotpath`` to use it.
"""
from . import data  # noqa: F401
