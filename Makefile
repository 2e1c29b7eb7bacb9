# Builds the gfx950 engine (C ABI) and the oracle's optional native bits.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
SRC := $(wildcard pycsou_amd/csrc/*.hip)
HDR := $(wildcard pycsou_amd/csrc/*.hpp) include/pycsou_hip.h
LIB := pycsou_amd/lib/libpycsou_hip.so
OBJ := $(patsubst pycsou_amd/csrc/%.hip,build/%.o,$(SRC))
FLAGS := --offload-arch=$(ARCH) -O3 -fno-slp-vectorize -fPIC -std=c++17 -Wall -Wno-unused-function -Iinclude

all: $(LIB)

build/%.o: pycsou_amd/csrc/%.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(FLAGS) $(FLAGS_$*) -c $< -o $@

$(LIB): $(OBJ)
	@mkdir -p pycsou_amd/lib
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJ) -L/opt/rocm/lib -lrocfft -Wl,-rpath,/opt/rocm/lib

clean:
	rm -rf build $(LIB)

.PHONY: all clean

# Diagnostic build with s_memtime stamps in the march kernel (tools/march_stamps.py)
STAMP_LIB := pycsou_amd/lib/diag/libpycsou_hip.so
stamps: $(SRC) $(HDR)
	@mkdir -p pycsou_amd/lib/diag
	$(HIPCC) $(FLAGS) -DPCS_STAMPS -shared -o $(STAMP_LIB) $(SRC) -L/opt/rocm/lib -lrocfft
.PHONY: stamps
