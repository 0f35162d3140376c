# Build of the MI355X (gfx950) MacroC hot path: one shared library with a C ABI.
# -ffp-contract=off keeps every product/sum rounded as written (bit-parity with the oracle).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CXXFLAGS ?= -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=$(ARCH) -Wall -Wno-unused-function
SRC = macroc_amd/csrc/api.cpp macroc_amd/csrc/dmda.cpp macroc_amd/csrc/comm.cpp macroc_amd/csrc/vtu.cpp \
      macroc_amd/csrc/kernels.hip
HDR = macroc_amd/csrc/mcx_internal.h include/macroc_amd.h
LIB = macroc_amd/libmacroc_amd.so
OBJ = $(patsubst macroc_amd/csrc/%,build/%.o,$(SRC))

all: $(LIB) oracle driver

build/%.o: macroc_amd/csrc/% $(HDR)
	@mkdir -p build
	$(HIPCC) $(CXXFLAGS) -c $< -o $@

$(LIB): $(OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJ) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

driver: macroc_amd/driver/macroc_amd
macroc_amd/driver/macroc_amd: macroc_amd/driver/main.c include/macroc_amd.h $(LIB)
	gcc -O2 -std=gnu11 -Iinclude -o $@ macroc_amd/driver/main.c -Lmacroc_amd -lmacroc_amd -Wl,-rpath,'$$ORIGIN/..'

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf build $(LIB) macroc_amd/driver/macroc_amd
	$(MAKE) -s -C oracle clean

.PHONY: all oracle driver clean
