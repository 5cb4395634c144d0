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

all: $(LIB) oracle

build/%.o: redisson_amd/csrc/%.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# -z now: every HIP/RCCL symbol is bound when the library loads.  Lazily bound
# calls made after `import torch` (which brings its own libamdhip64 into the
# global symbol scope) would otherwise resolve to torch's HIP runtime, which
# does not know these kernels (hipOccupancyMaxActiveBlocksPerMultiprocessor
# answered 1 there: persistent grids a third of their size).
$(LIB): $(OBJ)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(OBJ) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -Wl,-z,now

oracle:
	$(MAKE) -s -C oracle

asm: $(SRC)
	@mkdir -p build/asm
	for f in $(SRC); do $(HIPCC) $(HIPFLAGS) -S --cuda-device-only -o build/asm/$$(basename $$f .hip).s $$f; done

clean:
	rm -rf build $(LIB)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean asm
