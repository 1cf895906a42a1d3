# Top-level build: the HIP product library, the C-ABI test harness and the
# oracle.  hipcc cross-compiles gfx950 code objects without a GPU.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
JOBS ?= 8

SRC := catears_amd/csrc
# EXPERIMENTS=1: the measurement build for tools/ -- every tuning variant and
# the DIAG ablation kernels (wrong results, timing only) -- as a separate
# library (point CATEARS_HIP_LIB at it).  The product library carries the
# default kernels and the documented, bit-identical alternatives only.
EXPERIMENTS ?= 0
ifeq ($(EXPERIMENTS),1)
OBJ := build/obj_exp
LIB := catears_amd/lib/libcatears_hip_exp.so
EXPFLAGS := -DCATEARS_EXPERIMENTS -DCATEARS_DIAG
else
OBJ := build/obj
LIB := catears_amd/lib/libcatears_hip.so
EXPFLAGS :=
endif

# -ffp-contract=off: the reference's float arithmetic is never fused
# (x86-64 without FMA); keeping mul/add separate makes the fbank, CMVN and
# epilogue arithmetic bit-identical to it.  MFMA accumulation is unaffected.
# No packed-FP32 VALU (v_pk_add/mul/fma_f32, v_pk_mov_b32) in any kernel:
# under concurrent MFMA kernels on the same CUs their results in lanes 48-63
# were wrong in ~2 % of fast-fbank launches, and with the feature off in none
# (tools/experiments/lds_race_stress.py).  The host-side cc1
# prints "not a recognized feature" for it and ignores it.
NOPK := -Xclang -target-feature -Xclang -packed-fp32-ops
HIPFLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -ffp-contract=off \
            -Iinclude -I$(SRC) -Wall -Wno-unused-function $(NOPK) $(EXPFLAGS)
CXX ?= g++
HOSTFLAGS := -O2 -fPIC -std=c++17 -ffp-contract=off -Iinclude -I$(SRC) -I/opt/rocm/include \
             -D__HIP_PLATFORM_AMD__ -Wall $(EXPFLAGS)

KERNELS := $(wildcard $(SRC)/kernels/*.hip)
HOSTSRC := $(SRC)/capi.cc $(SRC)/tables.cc $(SRC)/model_io.cc
OBJS := $(patsubst $(SRC)/kernels/%.hip,$(OBJ)/%.o,$(KERNELS)) \
        $(patsubst $(SRC)/%.cc,$(OBJ)/%.o,$(HOSTSRC))
HDRS := include/catears_gpu.h $(SRC)/internal.h $(SRC)/model_io.h $(SRC)/fbank_ops.h $(SRC)/fbank8_ops.h $(SRC)/tile_order.h $(SRC)/lds_dma.h

all: $(LIB) oracle

# `make EXPERIMENTS=1 lib` builds only the measurement library
lib: $(LIB)

# the bf16x6 GEMM's small per-lane arrays stay in registers (hipcc would
# otherwise promote one into LDS at 1 block/CU: +36 KB of LDS traffic)
$(OBJ)/gemm_bf16x6.o $(OBJ)/gemm_f16x3.o: HIPFLAGS += -mllvm -disable-promote-alloca-to-lds=1
# no SLP-packed v_pk_add_f32 beside MFMAs (MI355X_MICROARCH.md: packed f32
# VALU costs more issue cycles than the scalar pair in an MFMA gap)
$(OBJ)/gemm_bf16x6.o: HIPFLAGS += -fno-slp-vectorize $(X6FLAGS)

# the exact fbank kernel holds a frame's FFT in 64 registers per lane: the
# SLP vectorizer's packed f32 pairs cost it ~20 registers of shuffles and
# pushed it into scratch
$(OBJ)/fbank.o $(OBJ)/fbank_nocase.o: HIPFLAGS += -fno-slp-vectorize
$(OBJ)/fbank_nocase.o: $(SRC)/kernels/fbank.hip

# CMVNFLAGS: experiment defines for the CMVN kernel (e.g. -DCMVN_TILE=48)
$(OBJ)/cmvn.o: HIPFLAGS += $(CMVNFLAGS)

# the fast fbank mode (fbank.hip's lane program again) is not bit-exact by
# design: let it contract mul/add
$(OBJ)/fbank_fma.o: HIPFLAGS += -ffp-contract=fast -fno-slp-vectorize
$(OBJ)/fbank_fma.o: $(SRC)/kernels/fbank.hip

$(OBJ)/%.o: $(SRC)/kernels/%.hip $(HDRS) Makefile
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJ)/%.o: $(SRC)/%.cc $(HDRS)
	@mkdir -p $(OBJ)
	$(CXX) $(HOSTFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	@mkdir -p $(dir $(LIB))
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -Wl,--no-undefined

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf build $(LIB) catears_amd/lib/libcatears_hip_exp.so $(PKLIB) $(PKTEST)
	$(MAKE) -C oracle clean

.PHONY: all lib oracle clean

# ---------------------------------------------------------------------------
# Drop-in pocketkaldi classes (C++ host layer over the C-ABI).  compat/ holds
# stand-ins for the reference's container headers, used only when building
# outside the reference tree (a reference build finds its own first).
HOST := catears_amd/host
PKLIB := catears_amd/lib/libcatears_pk.so
PKINC := -I$(HOST)/include -I$(HOST)/compat -Iinclude -I/opt/rocm/include
PKFLAGS := -O2 -fPIC -std=c++17 -ffp-contract=off -D__HIP_PLATFORM_AMD__ -Wall $(PKINC)
PKSRC := $(wildcard $(HOST)/src/*.cc) $(wildcard $(HOST)/compat_src/*.cc)
PKOBJS := $(patsubst $(HOST)/%.cc,$(OBJ)/host/%.o,$(PKSRC))
PKHDRS := $(wildcard $(HOST)/include/*.h) $(wildcard $(HOST)/compat/*.h) include/catears_gpu.h
PKTEST := catears_amd/lib/pk_dropin

$(OBJ)/host/%.o: $(HOST)/%.cc $(PKHDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(PKFLAGS) -c $< -o $@

$(PKLIB): $(PKOBJS) $(LIB)
	$(CXX) -shared -o $@ $(PKOBJS) -Lcatears_amd/lib -lcatears_hip -L/opt/rocm/lib -lamdhip64 \
	    -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,/opt/rocm/lib -Wl,--no-undefined

$(PKTEST): tests/native/pk_dropin.cc $(PKLIB) $(PKHDRS)
	$(CXX) $(PKFLAGS) -rdynamic -o $@ $< -Lcatears_amd/lib -lcatears_pk -lcatears_hip -L/opt/rocm/lib -lamdhip64 \
	    -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,/opt/rocm/lib

COMPATTEST := build/bin/compat_test
$(COMPATTEST): tests/native/compat_test.cc $(wildcard $(HOST)/compat_src/*.cc) $(wildcard $(HOST)/compat/*.h)
	@mkdir -p $(dir $@)
	$(CXX) -O1 -std=c++17 -Wall -I$(HOST)/compat -o $@ $< $(wildcard $(HOST)/compat_src/*.cc)

# The same container layer and the model-file parsers under AddressSanitizer +
# UndefinedBehaviorSanitizer (host code only; tests/test_dropin.py runs them
# on the CPU): compat_test, and parse_fuzz over model_io.cc (the C-ABI's NN02 /
# MAT0 / VEC0 / config readers) and the drop-in Nnet::Read, fed truncated and
# corrupted images.  The drop-in nnet.cc links the product libraries for the
# device calls it never makes here.
SANFLAGS := -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all
COMPATASAN := build/bin/compat_test_asan
FUZZASAN := build/bin/parse_fuzz_asan
$(COMPATASAN): tests/native/compat_test.cc $(wildcard $(HOST)/compat_src/*.cc) $(wildcard $(HOST)/compat/*.h)
	@mkdir -p $(dir $@)
	$(CXX) $(SANFLAGS) -std=c++17 -Wall -I$(HOST)/compat -o $@ $< $(wildcard $(HOST)/compat_src/*.cc)
$(FUZZASAN): tests/native/parse_fuzz.cc $(SRC)/model_io.cc $(SRC)/model_io.h $(HOST)/src/nnet.cc $(PKHDRS) $(LIB) \
             $(wildcard $(HOST)/compat_src/*.cc)
	@mkdir -p $(dir $@)
	$(CXX) $(SANFLAGS) -std=c++17 -ffp-contract=off -D__HIP_PLATFORM_AMD__ -Wall $(PKINC) -I$(SRC) -o $@ \
	    tests/native/parse_fuzz.cc $(SRC)/model_io.cc $(HOST)/src/nnet.cc $(HOST)/src/runtime.cc \
	    $(HOST)/src/linalg.cc $(wildcard $(HOST)/compat_src/*.cc) \
	    -Lcatears_amd/lib -lcatears_hip -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,$(CURDIR)/catears_amd/lib \
	    -Wl,-rpath,/opt/rocm/lib
sanitize: $(COMPATASAN) $(FUZZASAN)
.PHONY: sanitize

host: $(PKLIB) $(PKTEST) $(COMPATTEST)
all: host
.PHONY: host
