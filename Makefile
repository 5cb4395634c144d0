# librsketch.so: the gfx950 sketch engine (HIP kernels + C ABI), built in-tree
# so it travels to the GPU box with the repo snapshot.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
# -ffp-contract=off: the PFCOUNT estimator must not fuse into FMAs (Redis on
# x86-64 gcc -O2 has none); integer paths are unaffected.
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -ffp-contract=off -Wall -Wno-unused-result
SRC := $(wildcard redisson_amd/csrc/*.hip)
HDR := $(wildcard redisson_amd/csrc/*.h) $(wildcard include/*.h)
OBJ := $(patsubst redisson_amd/csrc/%.hip,build/%.o,$(SRC))
LIB := redisson_amd/librsketch.so
# The test / bench support library (include/rsketch_diag.h): generators,
# microbenchmarks, tuning variants, route overrides.  Not linked to the
# product library; it shares only the internal headers.
DSRC := $(wildcard redisson_amd/csrc/diag/*.hip)
DHDR := $(HDR) $(wildcard redisson_amd/csrc/diag/*.h)
DOBJ := $(patsubst redisson_amd/csrc/diag/%.hip,build/diag/%.o,$(DSRC))
DLIB := redisson_amd/librsketch_diag.so

all: $(LIB) $(DLIB) oracle

# Product objects: hidden visibility, so the library exports exactly the C ABI
# of include/rsketch.h (its declarations carry default visibility).
build/%.o: redisson_amd/csrc/%.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -fvisibility=hidden -fvisibility-inlines-hidden -c $< -o $@

build/diag/%.o: redisson_amd/csrc/diag/%.hip $(DHDR)
	@mkdir -p build/diag
	$(HIPCC) $(HIPFLAGS) -fvisibility=hidden -fvisibility-inlines-hidden -c $< -o $@

$(DLIB): $(DOBJ)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(DOBJ) -L/opt/rocm/lib -lrccl -lhsa-runtime64 -Wl,-rpath,/opt/rocm/lib -Wl,-z,now

# -z now: every HIP/RCCL symbol is bound when the library loads.  Lazily bound
# calls made after `import torch` (which brings its own libamdhip64 into the
# global symbol scope) would otherwise resolve to torch's HIP runtime, which
# does not know these kernels (hipOccupancyMaxActiveBlocksPerMultiprocessor
# answered 1 there: persistent grids a third of their size).
$(LIB): $(OBJ)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(OBJ) -L/opt/rocm/lib -lrccl -lhsa-runtime64 -Wl,-rpath,/opt/rocm/lib -Wl,-z,now

oracle:
	$(MAKE) -s -C oracle

asm: $(SRC)
	@mkdir -p build/asm
	for f in $(SRC) $(DSRC); do $(HIPCC) $(HIPFLAGS) -S --cuda-device-only -o build/asm/$$(basename $$f .hip).s $$f; done

clean:
	rm -rf build $(LIB) $(DLIB)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean asm
