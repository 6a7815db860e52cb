# Build for MI355X (gfx950) only. Outputs stay in-tree so they travel to the GPU box with gpurun.
#   make            -> genomicsbench_palisade_amd/lib/libgb.so (C ABI: gb_*), libgkl_pairhmm_c.so
#                      (reference-compatible drop-in), bin/phmm, oracle/_build/liboracle.so
#   make ref        -> also oracle/_ref/* (reference kernels; needs /root/reference)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
PKG := genomicsbench_palisade_amd
CSRC := $(PKG)/csrc
LIB := $(PKG)/lib
BIN := $(PKG)/bin
# -ffp-contract=off is part of the arithmetic contract (no FMA anywhere).
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -Wall -Wno-unused-result
HOSTCXX := g++
HOSTFLAGS := -O3 -std=c++17 -fPIC -ffp-contract=off -Wall

HIP_SRCS := $(wildcard $(CSRC)/*.hip)
HIP_OBJS := $(patsubst $(CSRC)/%.hip,$(LIB)/obj/%.o,$(HIP_SRCS)) $(LIB)/obj/gb_common.o
HDRS := $(wildcard include/*.h) $(wildcard $(CSRC)/*.h)

.PHONY: all ref clean oracle
DROPINS := $(LIB)/libgkl_pairhmm_c.so $(LIB)/libgb_chain_dropin.so $(LIB)/libgb_bsw_dropin.so $(LIB)/libgb_fmi_dropin.so
all: $(LIB)/libgb.so $(DROPINS) $(BIN)/phmm $(BIN)/chain $(BIN)/bsw $(BIN)/fmi oracle tests/_build/fmi_class_driver \
     tests/_build/libdropin_bench.so tests/_build/liblds_poison.so

# the latency-bound DP loops schedule better for instruction-level parallelism (chain_rows -1.8 %,
# phmm +0.8 %, bsw / fmi neutral; profiles/r04zb_sched_ab.log)
$(LIB)/obj/chain_rows.o $(LIB)/obj/phmm.o: HIPFLAGS += -mllvm -amdgpu-sched-strategy=max-ilp

# the Makefile itself is a prerequisite: flag changes (the per-object scheduler flags above) rebuild
$(LIB)/obj/%.o: $(CSRC)/%.hip $(HDRS) Makefile
	@mkdir -p $(LIB)/obj
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB)/obj/gb_common.o: $(CSRC)/gb_common.cpp $(HDRS) Makefile
	@mkdir -p $(LIB)/obj
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(LIB)/libgb.so: $(HIP_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(HIP_OBJS) -L/opt/rocm/lib -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib

# Reference-compatible drop-in: exports initPairHMM()/computelikelihoodsboth() with the reference's
# C++ linkage (IntelPairHmmCSource.cpp:29-115) on top of libgb.so.
$(LIB)/libgkl_pairhmm_c.so: $(CSRC)/gkl_dropin.cpp $(LIB)/libgb.so $(HDRS)
	$(HOSTCXX) $(HOSTFLAGS) -shared -o $@ $< -L$(LIB) -lgb -Wl,-rpath,'$$ORIGIN'

# host_chain_kernel (C++ linkage, gb_compat/minimap2_chain.h) and BandedPairWiseSW (gb_compat/bandedSWA.h)
$(LIB)/libgb_%_dropin.so: $(CSRC)/%_dropin.cpp $(LIB)/libgb.so $(HDRS) $(wildcard include/gb_compat/*.h)
	$(HOSTCXX) $(HOSTFLAGS) -shared -o $@ $< -L$(LIB) -lgb -Wl,-rpath,'$$ORIGIN'

$(BIN)/chain: $(PKG)/drivers/chain_main.cpp $(LIB)/libgb_chain_dropin.so
	@mkdir -p $(BIN)
	$(HOSTCXX) $(HOSTFLAGS) -o $@ $< -L$(LIB) -lgb_chain_dropin -lgb -Wl,-rpath,'$$ORIGIN/../lib'

$(BIN)/bsw: $(PKG)/drivers/bsw_main.cpp $(LIB)/libgb_bsw_dropin.so
	@mkdir -p $(BIN)
	$(HOSTCXX) $(HOSTFLAGS) -o $@ $< -L$(LIB) -lgb_bsw_dropin -lgb -Wl,-rpath,'$$ORIGIN/../lib'

$(BIN)/fmi: $(PKG)/drivers/fmi_main.cpp $(LIB)/libgb.so
	@mkdir -p $(BIN)
	$(HOSTCXX) $(HOSTFLAGS) -o $@ $< -L$(LIB) -lgb -lz -Wl,-rpath,'$$ORIGIN/../lib'

$(BIN)/phmm: $(PKG)/drivers/phmm_main.cpp $(LIB)/libgb.so
	@mkdir -p $(BIN)
	$(HOSTCXX) $(HOSTFLAGS) -pthread -o $@ $< -L$(LIB) -lgb -Wl,-rpath,'$$ORIGIN/../lib'

# test driver: benchmarks/fmi/fmi.cpp's batch loop over the FMI_search class (tests/test_fmi_dropin.py)
tests/_build/fmi_class_driver: tests/cpp/fmi_class_driver.cpp $(LIB)/libgb_fmi_dropin.so include/gb_compat/FMI_search.h
	@mkdir -p tests/_build
	$(HOSTCXX) $(HOSTFLAGS) -o $@ $< -L$(LIB) -lgb_fmi_dropin -lgb -Wl,-rpath,'$$ORIGIN/../../$(LIB)'

# bench harness: host_chain_kernel / getScores16 called the way the reference benchmarks call them
tests/_build/libdropin_bench.so: tests/cpp/dropin_bench.cpp $(LIB)/libgb_chain_dropin.so $(LIB)/libgb_bsw_dropin.so $(wildcard include/gb_compat/*.h)
	@mkdir -p tests/_build
	$(HOSTCXX) $(HOSTFLAGS) -pthread -shared -o $@ $< -L$(LIB) -lgb_chain_dropin -lgb_bsw_dropin -lgb -Wl,-rpath,'$$ORIGIN/../../$(LIB)'

# test infrastructure: fills every CU's LDS with adversarial patterns (tests/test_lds_poison.py)
tests/_build/liblds_poison.so: tests/cpp/lds_poison.hip
	@mkdir -p tests/_build
	$(HIPCC) --offload-arch=$(ARCH) -O2 -std=c++17 -fPIC -shared -o $@ $<

oracle:
	$(MAKE) -s -C oracle all

ref:
	$(MAKE) -s -C oracle ref

clean:
	rm -rf $(LIB) $(BIN)
	$(MAKE) -s -C oracle clean
