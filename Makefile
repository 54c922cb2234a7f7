# Native build of the MI355X path tracer.  `make` (or __graft_entry__.build()) builds in-tree:
#   pathtracercuda_amd/lib/libpt_hip.so   HIP kernels + device C ABI (include/pt_hip.h), gfx950
#   pathtracercuda_amd/lib/libpt_host.so  host C++ layer + C ABI (include/pathtracer_amd.hpp, pt_host.h)
#   pathtracercuda_amd/lib/pathtracer     CLI (reference main.cpp headless path)
#   pathtracercuda_amd/lib/fp_exhaustive  all-inputs check of the kernel's fast 1/x and sqrt (GPU)
#   pathtracercuda_amd/lib/host_sanitize_check  ASan/UBSan mutation check of the host parsers (CPU)
#   oracle/liboracle.so                   CPU restatement (test infrastructure only)
# Every FP unit is built with -ffp-contract=off: the GPU result is compared bit for bit with the
# oracle, and the host-built BVH / transforms / camera feed the GPU directly.
HIPCC ?= /opt/rocm/bin/hipcc
CXX ?= g++
ARCH ?= gfx950
LIB := pathtracercuda_amd/lib
SRC := pathtracercuda_amd/csrc
HOST_SRCS := $(SRC)/host/math_camera.cpp $(SRC)/host/hittable.cpp $(SRC)/host/bvh_build.cpp \
             $(SRC)/host/json_min.cpp $(SRC)/host/scene_json.cpp $(SRC)/host/image_io.cpp \
             $(SRC)/host/renderer.cpp $(SRC)/host/host_capi.cpp
HOST_HDRS := include/pathtracer_amd.hpp include/pt_host.h include/pt_hip.h $(SRC)/host/host_internal.h $(SRC)/host/json_min.h

# -fno-slp-vectorize: the kernel's packed FP32 pairs are written out (ext_vector_type); the SLP
# vectorizer's own pairings bound two scalars of the GGX visibility term into one register tuple
# that the allocator then spilled around a range guard in every GGX shading.  Off: scratch 40 -> 12
# B/lane (no spill inside the loop), +4.6 % on C3 same-box (profiles/r03_slp_ab.json).
HIPFLAGS ?= --offload-arch=$(ARCH) -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -fPIC -fvisibility=hidden \
            -mcode-object-version=5 -Iinclude -Wall -Wno-unused-result
CXXFLAGS ?= -O2 -std=c++17 -ffp-contract=off -fno-fast-math -fPIC -Iinclude -I$(SRC)/host -Wall -Wextra \
            -Wno-unused-parameter -Wno-missing-field-initializers

all: $(LIB)/libpt_hip.so $(LIB)/libpt_host.so $(LIB)/pathtracer $(LIB)/fp_exhaustive $(LIB)/host_sanitize_check oracle

$(LIB):
	mkdir -p $(LIB)

$(LIB)/libpt_hip.so: $(SRC)/pt_kernels.hip $(wildcard $(SRC)/*.h) include/pt_hip.h | $(LIB)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(SRC)/pt_kernels.hip -lrccl

$(LIB)/libpt_host.so: $(HOST_SRCS) $(HOST_HDRS) $(LIB)/libpt_hip.so
	$(CXX) $(CXXFLAGS) -shared -o $@ $(HOST_SRCS) -L$(LIB) -lpt_hip -lz -Wl,-rpath,'$$ORIGIN'

$(LIB)/pathtracer: $(SRC)/host/cli_main.cpp $(LIB)/libpt_host.so
	$(CXX) $(CXXFLAGS) -o $@ $(SRC)/host/cli_main.cpp -L$(LIB) -lpt_host -lpt_hip -lpthread -Wl,-rpath,'$$ORIGIN'

$(LIB)/fp_exhaustive: tools/fp_exhaustive.hip $(SRC)/pt_math.h | $(LIB)
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -ffp-contract=off -o $@ tools/fp_exhaustive.hip

oracle:
	$(MAKE) -C oracle

# CPU-only sanitizer build of the host parsers (scene JSON, RGBE/PNG decode, BVH build) with a
# mutation driver; run by tests/test_host.py.  Links libpt_hip.so for the symbols only (no GPU call).
SAN_SRCS := $(filter-out $(SRC)/host/host_capi.cpp,$(HOST_SRCS))
$(LIB)/host_sanitize_check: tools/host_sanitize_check.cpp $(SAN_SRCS) $(HOST_HDRS) $(LIB)/libpt_hip.so
	$(CXX) -O1 -g -std=c++17 -ffp-contract=off -fsanitize=address,undefined -fno-sanitize-recover=undefined \
	  -fno-omit-frame-pointer -Iinclude -I$(SRC)/host -o $@ tools/host_sanitize_check.cpp $(SAN_SRCS) \
	  -L$(LIB) -lpt_hip -lz -lpthread -Wl,-rpath,'$$ORIGIN'
sanitize: $(LIB)/host_sanitize_check

clean:
	rm -f $(LIB)/libpt_hip.so $(LIB)/libpt_host.so $(LIB)/pathtracer
	$(MAKE) -C oracle clean

.PHONY: all oracle clean sanitize

# `make -s print-HIPFLAGS`: the flags snapshot builds (tools/snap_rev.sh) reuse
print-%:
	@echo $($*)
