"""The C++ host adapters (difacto_amd/host: GpuLocalizer, GpuFMLoss, GpuSGDUpdater, StoreGPU,
GpuSGDLearner over the C-ABI) and their test driver tests/host/host_tests.cc, which restates
the reference's own gtests (localizer_test.cc, fm_loss_test.cc, sgd_learner_test.cc)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "host_tests")
DATA = os.path.join(ROOT, "tests", "golden", "rcv1_100.libsvm")


def test_host_adapters_build_and_link():
    """g++ builds the adapters against the C-ABI header alone and the binary resolves
    libdifacto_amd.so (no HIP headers, no torch in the host layer)."""
    subprocess.check_call(["make", "-s", "build/host_tests"], cwd=ROOT)
    out = subprocess.check_output(["ldd", BIN], text=True)
    assert "libdifacto_amd.so" in out and "not found" not in out
    syms = subprocess.check_output(["nm", "-D", "--undefined-only", BIN], text=True)
    for s in ("dfx_train_step", "dfx_localize", "dfx_fm_predict", "dfx_fm_calcgrad",
              "dfx_store_pull", "dfx_store_push", "dfx_store_save", "dfx_store_load"):
        assert s in syms, s


@pytest.mark.gpu
def test_host_adapters_reference_gtests():
    assert os.path.exists(BIN), "build/host_tests missing: run make"
    r = subprocess.run([BIN, DATA], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    print(r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL PASSED" in r.stdout
