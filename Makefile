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

HOSTBIN = build/host_tests
TRAINBIN = build/dfx_train
HOSTLIB = difacto_amd/host/gpu_adapters.cc difacto_amd/host/reader.cc
HOSTSRC = $(HOSTLIB) difacto_amd/host/dist_store.cc difacto_amd/host/split_learner.cc \
  tests/host/host_tests.cc
HOSTHDR = difacto_amd/host/iface.h difacto_amd/host/gpu_adapters.h difacto_amd/host/reader.h \
  difacto_amd/host/dist_host.h difacto_amd/host/dist_store.h difacto_amd/host/split_learner.h \
  include/difacto_amd.h include/difacto_amd_dist.h
HOSTFLAGS = -std=c++14 -O2 -Wall -pthread

READERBIN = build/reader_tests
GENBIN = build/gen_criteo
CONVBIN = build/dfx_convert
RBENCH = build/reader_bench

DISTLIB = difacto_amd/libdfx_dist.so

all: $(LIB) $(DISTLIB) oracle $(HOSTBIN) $(TRAINBIN) $(READERBIN) $(GENBIN) $(CONVBIN) $(RBENCH) \
  build/expf_check build/locbench

$(RBENCH): difacto_amd/host/reader.cc tools/reader_bench.cc difacto_amd/host/reader.h
	@mkdir -p build
	g++ $(HOSTFLAGS) -o $@ difacto_amd/host/reader.cc tools/reader_bench.cc

# the data converter (src/reader/converter.h): text formats -> rec (CompressedRowBlock RecordIO)
$(CONVBIN): difacto_amd/host/reader.cc difacto_amd/host/convert_main.cc difacto_amd/host/reader.h \
  difacto_amd/host/iface.h
	@mkdir -p build
	g++ $(HOSTFLAGS) -o $@ difacto_amd/host/reader.cc difacto_amd/host/convert_main.cc

$(GENBIN): tools/gen_criteo.cc
	@mkdir -p build
	g++ -O2 -o $@ $<

# the readers alone (CPU only: no libdifacto_amd)
$(READERBIN): difacto_amd/host/reader.cc tests/host/reader_tests.cc difacto_amd/host/reader.h \
  difacto_amd/host/iface.h
	@mkdir -p build
	g++ $(HOSTFLAGS) -o $@ difacto_amd/host/reader.cc tests/host/reader_tests.cc -ldl

# C++ host adapters (the reference's Loss/Updater/Store over the C-ABI) + their test driver;
# plain g++ against the C-ABI (the sharded store's exchange, dist_host.o, links RCCL)
$(HOSTBIN): $(HOSTSRC) $(HOSTHDR) build/obj/dist_host.o $(LIB) $(DISTLIB)
	@mkdir -p build
	g++ $(HOSTFLAGS) -o $@ $(HOSTSRC) build/obj/dist_host.o -Ldifacto_amd -ldifacto_amd -ldfx_dist \
	  -L/opt/rocm/lib -lrccl -lamdhip64 \
	  -Wl,-rpath,'$$ORIGIN/../difacto_amd' -Wl,-rpath,/opt/rocm/lib

# the sharded store's C++ driver (host code: HIP runtime API + RCCL, built by hipcc)
build/obj/dist_host.o: difacto_amd/host/dist_host.cc difacto_amd/host/dist_host.h include/difacto_amd.h
	@mkdir -p build/obj
	$(HIPCC) -std=c++17 -O2 -fPIC -Wall -c $< -o $@

# the training driver (src/main.cc + SGDLearner::RunScheduler): reader -> feeder -> fused step,
# or the sharded store over RCCL / loopback
$(TRAINBIN): $(HOSTLIB) difacto_amd/host/train_main.cc difacto_amd/host/split_learner.cc \
  $(HOSTHDR) difacto_amd/host/dist_host.h build/obj/dist_host.o $(LIB) $(DISTLIB)
	@mkdir -p build
	g++ $(HOSTFLAGS) -o $@ $(HOSTLIB) difacto_amd/host/train_main.cc \
	  difacto_amd/host/split_learner.cc build/obj/dist_host.o \
	  -Ldifacto_amd -ldifacto_amd -ldfx_dist -L/opt/rocm/lib -lrccl -lamdhip64 \
	  -Wl,-rpath,'$$ORIGIN/../difacto_amd' -Wl,-rpath,/opt/rocm/lib

# the multi-GPU split driver's C-ABI (include/difacto_amd_dist.h): host code (HIP runtime
# API + RCCL) over libdifacto_amd.so, loaded by difacto_amd/_lib.py beside it
$(DISTLIB): difacto_amd/host/split_host.cc difacto_amd/host/split_host.h \
  include/difacto_amd_dist.h include/difacto_amd.h $(LIB)
	g++ -std=c++17 -O2 -fPIC -Wall -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -shared -o $@ \
	  difacto_amd/host/split_host.cc -Ldifacto_amd -ldifacto_amd -L/opt/rocm/lib -lrccl -lamdhip64 \
	  -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,/opt/rocm/lib

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

oracle:
	$(MAKE) -s -C oracle

# measurement: the fused step's Localizer alone (links the library's internals)
build/locbench: tools/locbench.hip $(LIB) $(HDRS)
	@mkdir -p build
	$(HIPCC) --offload-arch=$(ARCH) -O2 -std=c++17 -Wno-unused-result -o $@ $< -Ldifacto_amd \
	  -ldifacto_amd -Wl,-rpath,'$$ORIGIN/../difacto_amd'

# test infrastructure: the device's expf (csrc/expf.h) against the host's glibc expf
build/expf_check: tools/expf_check.hip $(CSRC)/expf.h
	@mkdir -p build
	$(HIPCC) --offload-arch=$(ARCH) -O2 -ffp-contract=off -o $@ $<

clean:
	rm -rf build $(LIB) $(DISTLIB)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean
