# Build recipe for librm (HIP, gfx950), the CPU oracle and the headless driver.
#   make            -> librm.so + oracle + rm_frameloop
#   make librm      -> opengl-raymarching-in-compute-shader_amd/librm.so
#   make oracle     -> oracle/_build/librm_oracle.so (test infrastructure)
#   make goldens    -> oracle/_ref/gen_camera_goldens (needs /root/reference; container only)
# Built artefacts stay in-tree (git-ignored) so they travel to the GPU box.

HIPCC    ?= /opt/rocm/bin/hipcc
CC       ?= gcc
CXX      ?= g++
PKG      := opengl-raymarching-in-compute-shader_amd
CSRC     := $(PKG)/csrc
ARCH     ?= gfx950
# -ffp-contract=off: no FMA contraction (HIP's device default is 'fast'), so every
# float op is one IEEE op in source order; HIP keeps correctly-rounded f32
# sqrt/div by default (-fhip-fp32-correctly-rounded-divide-sqrt).
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off \
            -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-result
OFLAGS   := -std=c11 -O3 -ffp-contract=off -fno-fast-math -fopenmp -fPIC -Wall -Wextra

LIBRM    := $(PKG)/librm.so
ORACLE   := oracle/_build/librm_oracle.so
DRIVER   := $(PKG)/rm_frameloop

RM_SRCS  := $(CSRC)/rm_api.hip $(CSRC)/rm_kernels.hip $(CSRC)/rm_table.hip $(CSRC)/rm_jit.hip $(CSRC)/rm_host.cpp $(CSRC)/rm_comm.cpp
RM_HDRS  := $(CSRC)/rm_scene.hpp $(CSRC)/rm_shard.hpp $(CSRC)/rm_fastmath.hpp $(CSRC)/rm_internal.hpp $(CSRC)/rm_jit.hpp $(CSRC)/rm_comm.hpp include/rm_api.h Makefile
# The table kernel's sources, embedded in librm.so for hiprtc (rm_jit.hip), under
# the names they #include each other by.
JIT_SRCS := rm_table.hip=$(CSRC)/rm_table.hip rm_internal.hpp=$(CSRC)/rm_internal.hpp \
            rm_scene.hpp=$(CSRC)/rm_scene.hpp rm_shard.hpp=$(CSRC)/rm_shard.hpp \
            rm_fastmath.hpp=$(CSRC)/rm_fastmath.hpp \
            ../../include/rm_api.h=include/rm_api.h

.PHONY: all librm oracle driver goldens asan clean
all: librm oracle driver
librm: $(LIBRM)
oracle: $(ORACLE)
driver: $(DRIVER)

$(PKG)/build/%.o: $(CSRC)/%.hip $(RM_HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# rm_kernels.hip is built twice: k_pixel + k_unshard (rm_kernels.o),
# and k_sample alone (rm_kernels_aa.o), both without SLP vectorisation: pairing
# f32 adds / muls into packed v_pk_* ops costs register moves to form the pairs
# (k_sample: 3.9 % slower per cfg3 frame), and since round 3's issue-slot changes
# it makes k_pixel spill 9 VGPRs (32 B of scratch per lane; none without SLP,
# round 4).  Both at -O2, which measured 0.4-2 % faster than -O3 for each (round
# 3, profiles/r03_compiler_ab.txt).
KFLAGS   := $(HIPFLAGS) -O2 -fno-slp-vectorize
$(PKG)/build/rm_kernels.o: $(CSRC)/rm_kernels.hip $(RM_HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(KFLAGS) -DRM_KERNELS_PIXEL_ONLY -c $< -o $@

$(PKG)/build/rm_kernels_aa.o: $(CSRC)/rm_kernels.hip $(RM_HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(KFLAGS) -DRM_KERNELS_AA_ONLY -c $< -o $@

# the scene-table kernels without SLP vectorisation too (generic -2.7 %, the
# hiprtc-specialised ones get the same flag in rm_jit.hip: -6.5 % per cfg3 frame)
$(PKG)/build/rm_table.o: $(CSRC)/rm_table.hip $(RM_HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -fno-slp-vectorize -c $< -o $@

$(PKG)/build/rm_jit_src.inc: $(CSRC)/rm_table.hip $(RM_HDRS) $(PKG)/tools/embed_sources.py
	@mkdir -p $(dir $@)
	python3 $(PKG)/tools/embed_sources.py $@ $(JIT_SRCS)

$(PKG)/build/rm_jit.o: $(CSRC)/rm_jit.hip $(RM_HDRS) $(PKG)/build/rm_jit_src.inc
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -I$(PKG)/build -c $< -o $@

$(PKG)/build/rm_host.o: $(CSRC)/rm_host.cpp $(RM_HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -x c++ -c $< -o $@

# RCCL is bound at run time (dlopen, rm_comm.cpp): librm does not link it.
$(PKG)/build/rm_comm.o: $(CSRC)/rm_comm.cpp $(RM_HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(LIBRM): $(PKG)/build/rm_api.o $(PKG)/build/rm_kernels.o $(PKG)/build/rm_kernels_aa.o $(PKG)/build/rm_table.o $(PKG)/build/rm_jit.o $(PKG)/build/rm_host.o $(PKG)/build/rm_comm.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -lhiprtc -ldl

$(ORACLE): oracle/rm_oracle.c oracle/rm_oracle.h include/rm_api.h
	@mkdir -p $(dir $@)
	$(CC) $(OFLAGS) -shared -o $@ oracle/rm_oracle.c -lm

$(DRIVER): $(PKG)/tools/rm_frameloop.cpp include/rm/camera.hpp include/rm/input.hpp include/rm/texture.hpp $(LIBRM)
	$(CXX) -std=c++17 -O2 -Wall -Iinclude -o $@ $< -L$(PKG) -lrm -Wl,-rpath,'$$ORIGIN'

# Camera goldens from the reference's vendored GLM 0.9.8.5 (third-party, in
# /root/reference/includes/glm).  Output binary only under oracle/_ref/.
REF ?= /root/reference
goldens: oracle/_ref/gen_camera_goldens oracle/_ref/gen_input_goldens
	oracle/_ref/gen_camera_goldens > tests/golden/camera_goldens.json
	oracle/_ref/gen_input_goldens > tests/golden/input_goldens.json

oracle/_ref/gen_input_goldens: oracle/gen_input_goldens.cpp
	@mkdir -p oracle/_ref
	$(CXX) -std=c++11 -O2 -ffp-contract=off -I$(REF)/includes -o $@ $<

oracle/_ref/gen_camera_goldens: oracle/gen_camera_goldens.cpp
	@mkdir -p oracle/_ref
	$(CXX) -std=c++11 -O2 -ffp-contract=off -I$(REF)/includes -o $@ $<

# ---- host sanitizer build: CPU suite under ASan + UBSan ---------
# librm's host code (the C-ABI, the table compiler and its bounds, the uniform
# lookup, input replay, the shard map, the hiprtc driver) and the oracle, built
# with AddressSanitizer + UndefinedBehaviorSanitizer, every report fatal.  The
# sanitizers are on the host side only (-Xarch_host; the device code is the
# production build's): this build is for the CPU container, where no kernel runs
# anyway (GPU sanitizers are not available).  tests/test_sanitizers.py runs the
# host-logic CPU tests against it (LD_PRELOAD of clang's ASan runtime, RM_LIBRM,
# RM_ORACLE).
LLVM     ?= /opt/rocm/lib/llvm
ASAN_DIR := $(PKG)/build/asan
ASANLIB  := $(ASAN_DIR)/librm.so
ASANORC  := oracle/_build/librm_oracle_asan.so
SANHOST  := -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
            -Xarch_host -fno-sanitize-recover=all -Xarch_host -fno-omit-frame-pointer
SANFLAGS := -fsanitize=address,undefined -fno-sanitize-recover=all -fno-omit-frame-pointer
ASAN_OBJS := $(addprefix $(ASAN_DIR)/,rm_api.o rm_kernels.o rm_kernels_aa.o rm_table.o rm_jit.o rm_host.o rm_comm.o)
asan: $(ASANLIB) $(ASANORC)

$(ASAN_DIR)/%.o: $(CSRC)/%.hip $(RM_HDRS) $(PKG)/build/rm_jit_src.inc
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -O1 -g $(SANHOST) -I$(PKG)/build -c $< -o $@
$(ASAN_DIR)/rm_kernels.o: $(CSRC)/rm_kernels.hip $(RM_HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -O1 -g $(SANHOST) -DRM_KERNELS_PIXEL_ONLY -c $< -o $@
$(ASAN_DIR)/rm_kernels_aa.o: $(CSRC)/rm_kernels.hip $(RM_HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -O1 -g $(SANHOST) -DRM_KERNELS_AA_ONLY -c $< -o $@
$(ASAN_DIR)/rm_host.o: $(CSRC)/rm_host.cpp $(RM_HDRS)
	@mkdir -p $(dir $@)
	$(LLVM)/bin/clang++ -std=c++17 -O1 -g -fPIC -ffp-contract=off $(SANFLAGS) -c $< -o $@
$(ASAN_DIR)/rm_comm.o: $(CSRC)/rm_comm.cpp $(RM_HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -O1 -g $(SANHOST) -x hip -c $< -o $@
$(ASANLIB): $(ASAN_OBJS)
	$(LLVM)/bin/clang++ -shared -fPIC $(SANFLAGS) -shared-libsan -o $@ $^ -L/opt/rocm/lib -lamdhip64 -lhiprtc -ldl \
	  -Wl,-rpath,/opt/rocm/lib
$(ASANORC): oracle/rm_oracle.c oracle/rm_oracle.h include/rm_api.h
	@mkdir -p $(dir $@)
	$(LLVM)/bin/clang -std=c11 -O1 -g -ffp-contract=off -fno-fast-math -fopenmp -fPIC -Wall $(SANFLAGS) \
	  -shared -shared-libsan -o $@ oracle/rm_oracle.c -lm -L$(LLVM)/lib -Wl,-rpath,$(LLVM)/lib

clean:
	rm -rf $(PKG)/build $(LIBRM) $(DRIVER) oracle/_build oracle/_ref
