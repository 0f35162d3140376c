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

MPI_DIR ?= /opt/conda
MPI_FLAGS = -I$(MPI_DIR)/include -Wl,-rpath-link,/usr/lib/x86_64-linux-gnu $(MPI_DIR)/lib/libmpi.so -Wl,-rpath,$(MPI_DIR)/lib
TESTLAW = tests/libmcx_testlaw.so

all: $(LIB) oracle driver driver-mpi testlaw asan

build/%.o: macroc_amd/csrc/% $(HDR)
	@mkdir -p build
	$(HIPCC) $(CXXFLAGS) -c $< -o $@

$(LIB): $(OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJ) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

driver: macroc_amd/driver/macroc_amd
macroc_amd/driver/macroc_amd: macroc_amd/driver/main.c include/macroc_amd.h $(LIB)
	gcc -O2 -std=gnu11 -Iinclude -o $@ macroc_amd/driver/main.c -Lmacroc_amd -lmacroc_amd -Wl,-rpath,'$$ORIGIN/..'

# MPI build of the driver (one rank per GPU, like `mpirun -np N macroc`); skipped without MPICH
driver-mpi: macroc_amd/driver/macroc_amd_mpi
macroc_amd/driver/macroc_amd_mpi: macroc_amd/driver/main.c include/macroc_amd.h $(LIB)
	@if [ -f $(MPI_DIR)/include/mpi.h ]; then \
	  gcc -O2 -std=gnu11 -DMCX_WITH_MPI -Iinclude -o $@ macroc_amd/driver/main.c -Lmacroc_amd -lmacroc_amd \
	    -Wl,-rpath,'$$ORIGIN/..' $(MPI_FLAGS); \
	else echo "no MPI under $(MPI_DIR): driver-mpi skipped"; fi

# test fixture: an external constitutive law (device law + MicroPP-shaped host library) and the
# driver linked against it as against MicroPP (tests/test_gpu_callback.py)
testlaw: $(TESTLAW) tests/macroc_amd_micropp
$(TESTLAW): tests/csrc/testlaw.hip include/macroc_amd.h
	$(HIPCC) -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=$(ARCH) -shared -o $@ $<
tests/macroc_amd_micropp: macroc_amd/driver/main.c include/macroc_amd.h $(LIB) $(TESTLAW)
	gcc -O2 -std=gnu11 -DMCX_WITH_MICROPP -Iinclude -o $@ macroc_amd/driver/main.c -Lmacroc_amd -lmacroc_amd \
	  -Ltests -lmcx_testlaw -Wl,-rpath,'$$ORIGIN/../macroc_amd' -Wl,-rpath,'$$ORIGIN'

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf build $(LIB) macroc_amd/driver/macroc_amd macroc_amd/driver/macroc_amd_mpi $(TESTLAW) tests/macroc_amd_micropp
	$(MAKE) -s -C oracle clean

# Host sanitizer build: every library source with AddressSanitizer + UBSan on the
# host side only (-Xarch_host; device code is compiled as in the product build) linked with the C
# driver into one executable, and the oracle's CLI under the same sanitizers (gcc).  No GPU is
# touched: tests/test_asan.py runs the driver's -plan_only (mcx_plan / mcx_plan_halo: DMDA
# decomposition, halo plans) on 1-8 rank grids and the oracle's time loop, and fails on any
# sanitizer report.
ASAN_DIR = build/asan
ASAN_HOST = -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=all \
            -Xarch_host -fno-omit-frame-pointer
ASAN_OBJ = $(patsubst macroc_amd/csrc/%,$(ASAN_DIR)/%.o,$(SRC))
ASAN_EXE = $(ASAN_DIR)/macroc_amd_asan
ASAN_ORACLE = $(ASAN_DIR)/macroc_oracle_asan

asan: $(ASAN_EXE) $(ASAN_ORACLE)
$(ASAN_DIR)/%.o: macroc_amd/csrc/% $(HDR)
	@mkdir -p $(ASAN_DIR)
	$(HIPCC) -O1 -g -std=c++17 -fPIC -ffp-contract=off --offload-arch=$(ARCH) -Wall -Wno-unused-function $(ASAN_HOST) -c $< -o $@
$(ASAN_DIR)/main.c.o: macroc_amd/driver/main.c include/macroc_amd.h
	@mkdir -p $(ASAN_DIR)
	$(HIPCC) -x c -O1 -g -std=gnu11 -Iinclude $(ASAN_HOST) -c $< -o $@
$(ASAN_EXE): $(ASAN_OBJ) $(ASAN_DIR)/main.c.o
	$(HIPCC) --offload-arch=$(ARCH) $(ASAN_HOST) -o $@ $^ -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
$(ASAN_ORACLE): oracle/main.c oracle/oracle.c oracle/oracle.h
	@mkdir -p $(ASAN_DIR)
	gcc -O1 -g -ffp-contract=off -fopenmp -std=gnu11 -fsanitize=address,undefined -fno-sanitize-recover=all \
	  -fno-omit-frame-pointer -o $@ oracle/main.c oracle/oracle.c -lm

.PHONY: all oracle driver driver-mpi testlaw asan clean
