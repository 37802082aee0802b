# Build of the MI355X-native int8 path (hipcc only; no cmake needed).
#   dlq_amd/libdlq.so  -- the C-ABI library (include/dlq.h)
#   bin/dlq_e2e        -- the C++ launcher (reference infer_e2e.cu main)
#   bin/dlq_step       -- the per-step drivers (reference infer_conv1_bn1_relu / infer_layerN / infer_head)
#   oracle/            -- the CPU checker (test infrastructure; oracle/Makefile)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
# -ffp-contract=off: the fp32 epilogue/host-prep op order is part of the
# numerics contract (every fused multiply-add is an explicit fmaf).
HIPFLAGS = --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result
SRC = dlq_amd/csrc/kernels.hip dlq_amd/csrc/conv3x3.hip dlq_amd/csrc/conv3x3i.hip dlq_amd/csrc/conv3x3s2i.hip dlq_amd/csrc/block_l1.hip dlq_amd/csrc/stem.hip dlq_amd/csrc/head.hip dlq_amd/csrc/layerops.hip dlq_amd/csrc/gemm.hip dlq_amd/csrc/preproc.hip dlq_amd/csrc/fp8.hip dlq_amd/csrc/ref_f32.hip dlq_amd/csrc/capi.cpp dlq_amd/csrc/resnet18.cpp dlq_amd/csrc/mlp.cpp dlq_amd/csrc/wpack.cpp
HDR = include/dlq.h dlq_amd/csrc/dlq_internal.h dlq_amd/csrc/device_common.h

all: dlq_amd/libdlq.so bin/dlq_e2e bin/dlq_step tools/check/libplancap.so oracle

# the layer1 block interleaves its epilogue FMAs with MFMAs, and the convs'
# epilogues run beside the partner waves' MFMAs: keep their FMAs scalar
build/block_l1.o build/conv3x3i.o build/conv3x3s2i.o: HIPFLAGS += -fno-slp-vectorize

build/%.o: dlq_amd/csrc/%.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

build/%.o: dlq_amd/csrc/%.cpp $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -x hip -c -o $@ $<

dlq_amd/libdlq.so: build/kernels.o build/conv3x3.o build/conv3x3i.o build/conv3x3s2i.o build/block_l1.o build/stem.o build/head.o build/layerops.o build/gemm.o build/preproc.o build/fp8.o build/ref_f32.o build/capi.o build/resnet18.o build/mlp.o build/wpack.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^

bin/dlq_e2e: dlq_amd/csrc/main_e2e.cpp dlq_amd/libdlq.so include/dlq.h
	@mkdir -p bin
	$(HIPCC) $(HIPFLAGS) -x hip -o $@ $< -Ldlq_amd -ldlq -Wl,-rpath,'$$ORIGIN/../dlq_amd'

bin/dlq_step: dlq_amd/csrc/main_step.cpp dlq_amd/libdlq.so include/dlq.h
	@mkdir -p bin
	$(HIPCC) $(HIPFLAGS) -x hip -o $@ $< -Ldlq_amd -ldlq -Wl,-rpath,'$$ORIGIN/../dlq_amd'

# test infrastructure: the convs' LDS-DMA plans recorded by the kernels
# themselves (tests/test_gpu_dma_plan.py)
build/plancap%.o: tools/check/plan_capture.hip dlq_amd/csrc/conv3x3i.hip dlq_amd/csrc/conv3x3s2i.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -DPLANCAP_KIND=$* -I dlq_amd/csrc -c -o $@ $<

build/dmamask.o: tools/check/dma_mask_check.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -I dlq_amd/csrc -c -o $@ $<

tools/check/libplancap.so: build/plancap0.o build/plancap1.o build/dmamask.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf build bin dlq_amd/libdlq.so tools/check/libplancap.so
	$(MAKE) -C oracle clean

.PHONY: all oracle clean
