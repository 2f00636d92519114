# Builds libgym_amd.so (gfx950 HIP kernels behind the C ABI in include/gym_amd.h)
# in-tree, so the .so travels to the GPU box with the repo snapshot.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
SRC := $(wildcard gym_amd/csrc/*.hip)
OBJ := $(patsubst gym_amd/csrc/%.hip,build/%.o,$(SRC))
LIB := gym_amd/_lib/libgym_amd.so
HIPFLAGS := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -fvisibility=hidden -Wall -Wno-unused-function

.PHONY: all clean oracle asan variant
all: $(LIB)

build/%.o: gym_amd/csrc/%.hip gym_amd/csrc/ga_common.h gym_amd/csrc/adam_math.h include/gym_amd.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJ)
	@mkdir -p gym_amd/_lib
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(OBJ)

# ISA listing for inspection (register counts, MFMA/VALU mix).
build/%.s: gym_amd/csrc/%.hip
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) --cuda-device-only -S $< -o $@

clean:
	rm -rf build $(LIB)

# Diagnostic build with per-phase s_memtime stamps in the DeMo kernels (tools/demo_stamps.py).
STAMP_LIB := build/libgym_amd_stamps.so
stamps: $(STAMP_LIB)
$(STAMP_LIB): $(SRC) gym_amd/csrc/ga_common.h include/gym_amd.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -DGA_DEMO_STAMPS -shared -o $@ $(SRC)

# Host AddressSanitizer build of the C ABI: the argument validation and
# host wrappers of every ga_* entry point instrumented (-Xarch_host: the device code is
# built as usual; GPU sanitizers are not used).  tests/test_abi_asan.py loads it into a
# python run with the ASan runtime preloaded and drives test_abi.py's invalid-argument
# cases through it (no GPU needed).
ASAN_LIB := build/libgym_amd_asan.so
ASAN_RT := $(firstword $(wildcard /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so))
asan: $(ASAN_LIB)
$(ASAN_LIB): $(SRC) gym_amd/csrc/ga_common.h include/gym_amd.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer -shared-libsan \
		-shared -o $@ $(SRC)
	@echo "ASan runtime: $(ASAN_RT)"

# A kernel variant of the whole library for same-box A/B (tools/ab_lib.sh loads it
# through GYM_AMD_LIB): make variant VDEFS="-DSOME_FLAG=1" VNAME=name
VNAME ?= variant
VDEFS ?=
variant: build/libgym_amd_$(VNAME).so
build/libgym_amd_$(VNAME).so: $(SRC) gym_amd/csrc/ga_common.h include/gym_amd.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) $(VDEFS) -shared -o $@ $(SRC)
