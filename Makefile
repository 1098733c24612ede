# Builds libdifacto_amd.so (gfx950 HIP kernels + the C-ABI), the oracle (test
# infrastructure), and the C++ host adapters/tests.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
# -ffp-contract=off: the reference computes without FMA contraction; parity needs the same
HIPFLAGS = --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -ffp-contract=off -Wall -Wno-unused-function
CSRC = difacto_amd/csrc
OBJDIR = build/obj
SRCS = $(wildcard $(CSRC)/*.hip)
OBJS = $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.o,$(SRCS))
HDRS = $(wildcard $(CSRC)/*.h) include/difacto_amd.h
LIB = difacto_amd/libdifacto_amd.so

all: $(LIB) oracle

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf build $(LIB)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean
