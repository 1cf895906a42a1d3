# Top-level build: the HIP product library, the C-ABI test harness and the
# oracle.  hipcc cross-compiles gfx950 code objects without a GPU.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
JOBS ?= 8

SRC := catears_amd/csrc
OBJ := build/obj
LIB := catears_amd/lib/libcatears_hip.so

# -ffp-contract=off: the reference's float arithmetic is never fused
# (x86-64 without FMA); keeping mul/add separate makes the fbank, CMVN and
# epilogue arithmetic bit-identical to it.  MFMA accumulation is unaffected.
HIPFLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -ffp-contract=off \
            -Iinclude -I$(SRC) -Wall -Wno-unused-function
CXX ?= g++
HOSTFLAGS := -O2 -fPIC -std=c++17 -ffp-contract=off -Iinclude -I$(SRC) -I/opt/rocm/include \
             -D__HIP_PLATFORM_AMD__ -Wall

KERNELS := $(wildcard $(SRC)/kernels/*.hip)
HOSTSRC := $(SRC)/capi.cc $(SRC)/tables.cc
OBJS := $(patsubst $(SRC)/kernels/%.hip,$(OBJ)/%.o,$(KERNELS)) \
        $(patsubst $(SRC)/%.cc,$(OBJ)/%.o,$(HOSTSRC))
HDRS := include/catears_gpu.h $(SRC)/internal.h $(SRC)/fbank_ops.h

all: $(LIB) oracle

$(OBJ)/%.o: $(SRC)/kernels/%.hip $(HDRS)
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
	rm -rf build $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean
