# Builds the in-tree C-ABI library cubed_amd/libcubed_amd.so for gfx950.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CSRC := cubed_amd/csrc
STREAMS := $(foreach v,f32 f64 i64,$(CSRC)/stream_$(v).hip $(CSRC)/stream_$(v)_split.hip)
SRCS := $(CSRC)/fused.hip $(STREAMS) $(CSRC)/jit.hip $(CSRC)/copy_random.hip $(CSRC)/gemm_chain.hip
CPPSRCS := $(CSRC)/codec.cpp
OBJS := $(SRCS:.hip=.o) $(CPPSRCS:.cpp=.o)
HIPFLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -ffp-contract=off \
            -fhip-fp32-correctly-rounded-divide-sqrt -Wno-unused-result -Iinclude
LIB := cubed_amd/libcubed_amd.so

all: $(LIB) oracle

$(CSRC)/%.o: $(CSRC)/%.hip $(CSRC)/common.h $(CSRC)/vm.h $(CSRC)/fused_common.h $(CSRC)/kernels.h $(CSRC)/stream_impl.h include/cubed_amd.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/gemm_chain.o: $(CSRC)/gemm_bf16_w4l.h $(CSRC)/gemm_bf16_w4p.h $(CSRC)/gemm_f32_w4p.h

$(CSRC)/%.o: $(CSRC)/%.cpp include/cubed_amd.h
	g++ -O3 -fPIC -std=c++17 -Iinclude -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(OBJS) -o $@ -L/opt/rocm/lib -lhiprtc -lz -Wl,-rpath,/opt/rocm/lib

oracle:
	$(MAKE) -C oracle

clean:
	rm -f $(OBJS) $(LIB)

.PHONY: all clean oracle
