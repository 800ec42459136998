# Build of the MI355X-native Nori path_mis hot path.
#   make            product library (HIP kernels for gfx950 + host C++) and the oracle
#   make ref        reference-side checker binaries (pcg32 demo) from /root/reference sources
#   make clean
# Floating point: no contraction anywhere (the reference is built without FMA;
# SURVEY.md Appendix D shows contraction alone breaks 1e-4 parity), correctly
# rounded fp32 div/sqrt, denormals preserved.

HIPCC    ?= /opt/rocm/bin/hipcc
CXX      ?= g++
ARCH     ?= gfx950
PKG      := optix-renderer_amd
LIBDIR   ?= $(PKG)/lib
OBJDIR   ?= build/obj
JOBS     ?= 8

FP_FLAGS   := -ffp-contract=off -fno-fast-math
HOST_FLAGS := -std=c++17 -O2 -fPIC -Wall -Wextra -Wno-unused-parameter $(FP_FLAGS) -Iinclude -I$(PKG)/host -pthread
HIP_FLAGS  := -std=c++17 -O3 -fPIC --offload-arch=$(ARCH) $(FP_FLAGS) \
              -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero \
              -Iinclude -I$(PKG)/csrc -Wno-unused-result $(EXTRA_HIP)

HOST_SRC := $(PKG)/host/xml_lite.cpp $(PKG)/host/scene_loader.cpp $(PKG)/host/bvh_build.cpp $(PKG)/host/image_io.cpp \
            $(PKG)/host/png_decode.cpp $(PKG)/host/hdr_decode.cpp
HIP_SRC  := $(PKG)/csrc/nh_kernels.hip $(PKG)/csrc/nh_denoise.hip $(PKG)/csrc/nh_splat.hip $(PKG)/csrc/nh_api.hip
HOST_OBJ := $(patsubst $(PKG)/host/%.cpp,$(OBJDIR)/host_%.o,$(HOST_SRC))
# nh_wavefront.hip is compiled as four translation units (-DNH_WF_PART=k, each instantiating its own kernels) so
# its kernels build in parallel
WF_PARTS := 0 1 2 3
HIP_OBJ  := $(patsubst $(PKG)/csrc/%.hip,$(OBJDIR)/hip_%.o,$(HIP_SRC)) \
            $(foreach k,$(WF_PARTS),$(OBJDIR)/hip_nh_wavefront_p$(k).o)
HIP_DEPS := $(wildcard $(PKG)/csrc/*.h) include/nori_hip.h
# The wavefront kernels build without LLVM's machine-level LICM: it hoists loop invariants out of the traversal, bounce
# and tail loops into registers for the loop's whole length, which then spill (wf_tail_rr at 4 waves/SIMD: 448 ->
# 28 B/lane of scratch; wf_tail 256 -> 157 VGPRs; the persistent traversals 96 -> 88). C5 +3.6 %, other configs
# level; the splat TU keeps it (1 % faster with it). profiles/round6_ab_machine_licm.txt
WF_FLAGS := -mllvm -disable-machine-licm

LIB      := $(LIBDIR)/libnori_hip.so
HOSTLIB  := $(LIBDIR)/libnori_host.so
ORACLE   := oracle/_build/libnori_oracle.so
CLI      := $(LIBDIR)/nori_hip

RCPCHECK := tools/bin/rcp_exhaustive
VALUBENCH := tools/bin/valu_issue

MANUAL   := tests/c/bin/manual_scene

all: $(LIB) $(HOSTLIB) $(ORACLE) $(CLI) $(RCPCHECK) $(VALUBENCH) $(MANUAL)

# C test: a scene description filled field by field (no XML loader), rendered through the C-ABI and
# compared with the oracle (run by tests/test_gpu_parity.py)
$(MANUAL): tests/c/manual_scene.c $(LIB) $(ORACLE) include/nori_hip.h oracle/nori_oracle.h
	@mkdir -p tests/c/bin
	$(CC) -std=c99 -O2 -Wall -Iinclude -Ioracle -o $@ $< -L$(LIBDIR) -lnori_hip -Loracle/_build -lnori_oracle \
	    -lm -Wl,-rpath,'$$ORIGIN/../../../$(LIBDIR)' -Wl,-rpath,'$$ORIGIN/../../../oracle/_build'

# exhaustive check of the fast reciprocal the traversal kernels use (run by the GPU tests)
$(RCPCHECK): tools/rcp_exhaustive.hip $(HIP_DEPS)
	@mkdir -p tools/bin
	$(HIPCC) $(HIP_FLAGS) -o $@ $<

# VALU issue-rate microbenchmark (scripts/valu_issue.sh): the ceiling bench.py's limiter record divides by
$(VALUBENCH): tools/valu_issue.hip
	@mkdir -p tools/bin
	$(HIPCC) -std=c++17 -O3 --offload-arch=$(ARCH) -o $@ $<

$(OBJDIR)/host_%.o: $(PKG)/host/%.cpp $(wildcard $(PKG)/host/*.h) include/nori_hip.h
	@mkdir -p $(OBJDIR)
	$(CXX) $(HOST_FLAGS) -c $< -o $@

$(OBJDIR)/hip_nh_wavefront_p%.o: $(PKG)/csrc/nh_wavefront.hip $(HIP_DEPS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIP_FLAGS) $(WF_FLAGS) -DNH_WF_PART=$* -c $< -o $@

$(OBJDIR)/hip_%.o: $(PKG)/csrc/%.hip $(HIP_DEPS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIP_FLAGS) -c $< -o $@

# product library: host ingestion + HIP kernels + C ABI
$(LIB): $(HOST_OBJ) $(HIP_OBJ)
	@mkdir -p $(LIBDIR)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $^ -L/opt/rocm/lib -lrccl -lz -Wl,-rpath,/opt/rocm/lib

# host-only subset (scene loader, BVH builder, image I/O): usable without a GPU runtime
$(HOSTLIB): $(HOST_OBJ)
	@mkdir -p $(LIBDIR)
	$(CXX) -shared -fPIC -pthread -o $@ $^ -lz

$(CLI): $(PKG)/host/nori_hip_main.cpp $(LIB)
	$(CXX) $(HOST_FLAGS) -o $@ $< -L$(LIBDIR) -lnori_hip -Wl,-rpath,'$$ORIGIN'

# test infrastructure: CPU restatement of the reference path (never linked into the product)
$(ORACLE): oracle/nori_oracle.cpp oracle/nori_oracle.h include/nori_hip.h
	@mkdir -p oracle/_build
	$(CXX) -std=c++17 -O2 -fPIC -pthread $(FP_FLAGS) -Iinclude -Ioracle -shared -o $@ $<

ref:
	./oracle/build_ref.sh

clean:
	rm -rf build $(LIBDIR) oracle/_build oracle/_ref

.PHONY: all clean ref
