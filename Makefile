# Build of the MI355X (gfx950) ray tracer and its CPU checker.
#   make            -> product library + demo app + oracle library
#   make ref        -> oracle/_ref harness compiled against the reference's vendored glm
#                      (only where /root/reference exists; never on the GPU box)
ROCM      ?= /opt/rocm
HIPCC     ?= $(ROCM)/bin/hipcc
ARCH      ?= gfx950
PKG       := realtimeraytracing_gradproject_amd
SRC       := $(PKG)/csrc
LIBDIR    := $(PKG)/lib
BUILD     := build

# -ffp-contract=off everywhere on the path: the image is bit-compared with the oracle.
HIPFLAGS  := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function \
             -munsafe-fp-atomics
CXXFLAGS  := -O2 -std=c++17 -fPIC -ffp-contract=off -Wall
# Oracle: scalar C, explicit fmaf in the slab test (matches __builtin_fmaf on the GPU).
OCFLAGS   := -O2 -std=c11 -fPIC -ffp-contract=off -mfma -Wall -Wno-unused-function

# CPU baseline: the same restatement at -O3, scalar (no SIMD intrinsics; -mfma for the
# slab test's explicit fmaf; no errno, so sqrtf stays one instruction), counters compiled out, plain-compare
# min/max in the slab test (rt_oracle.c OMINF). Same frames as the checker. Bench-only, like the checker.
BCFLAGS   := -O3 -std=c11 -fPIC -ffp-contract=off -fno-math-errno -mfma -DORACLE_NO_COUNTERS

LIB       := $(LIBDIR)/librtamd.so
APP       := $(LIBDIR)/rt_app
ORACLE    := oracle/liboracle.so
BASELINE  := oracle/libbaseline.so
RCPCHECK  := tools/bin/recip_check
OCCPROBE  := tools/bin/occupancy_probe
CLKPROBE  := tools/bin/clock_probe
DSPPROBE  := tools/bin/libdispatch_probe.so

HDRS      := include/rt_api.h $(SRC)/rt_device.hpp $(SRC)/rt_internal.hpp $(SRC)/rt_trace_packet.inc

# Library variants with the non-default code-shape knobs still in the tree (rt_device.hpp / rt_trace.hip), each
# checked against the oracle on the GPU by tests/test_gpu_variants.py:
#   n1        RT_SHADOW_COMPACT=1 RT_HYBRID_T=8: workgroup shadow-ray compaction + per-lane subtree hand-off (the
#             north star's ballot / prefix-sum compaction designs)
#   n1root    RT_HYBRID_T=16 RT_HYBRID_ROOT=1: the hand-off considered at BLAS roots only
#   rays2     RT_PACKET_RAYS=2 RT_SAMPLE_LANES=0 RT_RCP_EXACT=0: two rays per lane (8 x 16 tiles), multi-sample
#             frames through the sample loop, IEEE divisions everywhere
#   alt       RT_PACKET_OCT=0 RT_REF_NOREFL=0 RT_RCP_EXACT=7 RT_MS_WIDE=1: min/max slab planes, the reflective REF
#             kernel for reflectivity 0, rcp + Newton everywhere, wide multi-sample tiles
#   wavetimes RT_WAVE_TIMES=1: the per-wave clock records of tools/wave_times.py
#   ldstop    RT_LDS_TOP=21: the largest BLAS's top two BFS levels staged in LDS per packet workgroup (the north
#             star's "LDS node packets", measured slower than the scalar-cache node loads: DESIGN §9)
VDIR      := $(LIBDIR)/variants
VSRCS     := $(SRC)/rt_api.cpp $(SRC)/rt_comm.cpp $(SRC)/rt_lbvh.hip $(SRC)/rt_trace.hip $(SRC)/rt_raster.hip \
             $(SRC)/rt_host.cpp $(HDRS) tools/build_variant.sh
VARIANTS  := n1 n1root rays2 alt wavetimes ldstop
VLIBS     := $(foreach v,$(VARIANTS),$(VDIR)/$(v)/librtamd.so)
DEFS_n1        := -DRT_SHADOW_COMPACT=1 -DRT_HYBRID_T=8
DEFS_n1root    := -DRT_HYBRID_T=16 -DRT_HYBRID_ROOT=1
DEFS_rays2     := -DRT_PACKET_RAYS=2 -DRT_SAMPLE_LANES=0 -DRT_RCP_EXACT=0
DEFS_alt       := -DRT_PACKET_OCT=0 -DRT_REF_NOREFL=0 -DRT_RCP_EXACT=7 -DRT_MS_WIDE=1
DEFS_wavetimes := -DRT_WAVE_TIMES=1
DEFS_ldstop    := -DRT_LDS_TOP=21

all: $(LIB) $(APP) $(ORACLE) $(BASELINE) $(RCPCHECK) $(OCCPROBE) $(CLKPROBE) $(DSPPROBE) $(VLIBS)

$(VDIR)/%/librtamd.so: $(VSRCS)
	bash tools/build_variant.sh $* $(DEFS_$*) > /dev/null

$(BUILD)/%.o: $(SRC)/%.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# The trace kernel without SLP vectorisation: packed v_pk_mul_f32 Moller-Trumbore products need their
# scalar triangle operands paired by s_mov (SALU, the kernel's tighter pipe) and VGPR pairs; scalar
# VALU reads the SGPRs directly (72 -> 58 VGPRs, C2 -4.6 %, C4 -4.2 %, C5 -4.6 %).
# Uniform regions left unstructurized: the walk's branches are wave-uniform (SCC / SGPR conditions), and the
# structurizer's flag registers and exec-mask glue around them cost SALU issue and SGPRs (C2's kernel 88 -> 84
# SGPRs, 59 -> 55 VGPRs; C2 / C3 / C4 -4 %, REF -1 %, C2F -2 %, frames bit-equal).
TRACEFLAGS := -fno-slp-vectorize -mllvm -structurizecfg-skip-uniform-regions=1
$(BUILD)/rt_trace.o: $(SRC)/rt_trace.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) $(TRACEFLAGS) -c $< -o $@

$(BUILD)/rt_api.o: $(SRC)/rt_api.cpp $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/rt_comm.o: $(SRC)/rt_comm.cpp $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/rt_host.o: $(SRC)/rt_host.cpp include/rt_api.h | $(BUILD)
	g++ $(CXXFLAGS) -c $< -o $@

$(LIB): $(BUILD)/rt_api.o $(BUILD)/rt_comm.o $(BUILD)/rt_host.o $(BUILD)/rt_lbvh.o $(BUILD)/rt_trace.o $(BUILD)/rt_raster.o | $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -ldl -Wl,-rpath,$(ROCM)/lib

$(APP): $(SRC)/host/rt_app.cpp $(wildcard $(SRC)/host/*.hpp) $(LIB) | $(LIBDIR)
	g++ $(CXXFLAGS) -I$(ROCM)/include -D__HIP_PLATFORM_AMD__ -o $@ $(SRC)/host/rt_app.cpp \
	    -L$(LIBDIR) -lrtamd -L$(ROCM)/lib -lamdhip64 -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,$(ROCM)/lib

$(ORACLE): oracle/rt_oracle.c oracle/rt_raster_oracle.c oracle/rt_oracle.h
	gcc $(OCFLAGS) -DORACLE_FLAGS='"$(OCFLAGS)"' -shared -o $@ oracle/rt_oracle.c oracle/rt_raster_oracle.c -lm -lpthread

$(BASELINE): oracle/rt_oracle.c oracle/rt_raster_oracle.c oracle/rt_oracle.h
	gcc $(BCFLAGS) -DORACLE_FLAGS='"$(BCFLAGS)"' -shared -o $@ oracle/rt_oracle.c oracle/rt_raster_oracle.c -lm -lpthread

ref:
	$(MAKE) -C oracle -f Makefile.ref

# exhaustive GPU check of rt::rcp_exact (the triangle test's 1 / det) against the IEEE division (tests/test_gpu_rcp.py)
$(RCPCHECK): tools/recip_check.hip $(SRC)/rt_device.hpp include/rt_api.h
	mkdir -p tools/bin
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -ffp-contract=off -o $@ $<

# resident waves per SIMD by register footprint (the wave-time traces' 7-wave ceiling)
$(OCCPROBE): tools/occupancy_probe.hip
	mkdir -p tools/bin
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -o $@ $<

# fabric traffic of the clock reads the tile balance's recording waves make
$(CLKPROBE): tools/clock_probe.hip
	mkdir -p tools/bin
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -o $@ $<

# one-workgroup kernels of k_tile_plan's shape and without its LDS / its 16 waves (tools/queue_probe.py)
$(DSPPROBE): tools/dispatch_probe.hip
	mkdir -p tools/bin
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -shared -fPIC -o $@ $<

$(BUILD) $(LIBDIR):
	mkdir -p $@

# Host sanitizer builds (ASan/UBSan for the oracle and the ingest; CPU only — GPU sanitizers are not
# available on this pool). build/asan/librtamd.so is the product library with its host C++ (rt_host.cpp: OBJ ingest,
# normals, camera, manipulator) compiled with -fsanitize=address,undefined, linked by g++ against the same HIP objects;
# build/asan/liboracle.so is the checker likewise. tools/asan_check.sh runs the CPU tests of those parts over them
# (RT_LIBRARY / ORACLE_LIBRARY, the gcc sanitizer runtimes preloaded into python).
ASAN      := $(BUILD)/asan
SANFLAGS  := -fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=undefined
asan: $(ASAN)/librtamd.so $(ASAN)/liboracle.so $(ASAN)/obj_ingest_fuzz

$(ASAN)/rt_host.o: $(SRC)/rt_host.cpp include/rt_api.h | $(ASAN)
	g++ -O1 -g -std=c++17 -fPIC -ffp-contract=off -Wall $(SANFLAGS) -c $< -o $@

$(ASAN)/librtamd.so: $(BUILD)/rt_api.o $(BUILD)/rt_comm.o $(ASAN)/rt_host.o $(BUILD)/rt_lbvh.o $(BUILD)/rt_trace.o $(BUILD)/rt_raster.o
	g++ -shared $(SANFLAGS) -o $@ $^ -L$(ROCM)/lib -lamdhip64 -ldl -Wl,-rpath,$(ROCM)/lib

$(ASAN)/liboracle.so: oracle/rt_oracle.c oracle/rt_raster_oracle.c oracle/rt_oracle.h | $(ASAN)
	gcc -O1 -g -std=c11 -fPIC -ffp-contract=off -mfma -Wall -Wno-unused-function $(SANFLAGS) \
	    -DORACLE_FLAGS='"asan"' -shared -o $@ oracle/rt_oracle.c oracle/rt_raster_oracle.c -lm -lpthread

# a standalone driver of the sanitized ingest over random and adversarial OBJ text (no Python in the process)
$(ASAN)/obj_ingest_fuzz: tools/obj_ingest_fuzz.cpp $(ASAN)/rt_host.o | $(ASAN)
	g++ -O1 -g -std=c++17 $(SANFLAGS) -o $@ $^

$(ASAN):
	mkdir -p $@

clean:
	rm -rf $(BUILD) $(LIB) $(APP) $(ORACLE) $(BASELINE) $(RCPCHECK) $(OCCPROBE) $(CLKPROBE) $(DSPPROBE) $(VDIR)

.PHONY: all clean ref asan
