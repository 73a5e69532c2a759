# Build for the MI355X-native framework (gfx950 / CDNA4).
#
# Parity with the reference makefile (/root/reference/makefile:1-15): the same targets `build`,
# `clean`, `run`, `runOn2` and the same product `./final` (stdin -> stdout). The toolchain is
# hipcc (device code, --offload-arch=gfx950) + g++ -fopenmp (host code, libgomp like PyTorch) +
# MPICH (/opt/conda) + RCCL, instead of mpicxx + nvcc + libcudart_static.
#
#   make build        libmoc.so (Python package) + ./final (MPI CLI)
#   make run          mpiexec -np 2 ./final < $(INPUT)
#   make runOn2       mpiexec -np 2 -machinefile mf --map-by node ./final < $(INPUT)
#   make test         CPU test-suite (pytest -m "not gpu")
#   make asan         ASan/UBSan build of the g++ host code -> ./final_asan (the thin hipcc launcher
#                     objects and all device code are built without sanitizers: no GPU ASan on the pool)
#   make tsan         ThreadSanitizer build of the host code -> ./final_tsan (OpenMP paths, CPU backend)

ROCM      ?= /opt/rocm
MPI_HOME  ?= /opt/conda
ARCH      ?= gfx950
HIPCC     ?= $(ROCM)/bin/hipcc
CXX       := g++
NP        ?= 2
INPUT     ?= tests/data/input1.txt
JOBS      ?= 8

BUILD     := build
OBJ       := $(BUILD)/obj
PKG_LIB   := mpi_openmp_cuda_amd/lib/libmoc.so
MPILIB    := $(BUILD)/mpilib

INC       := -Icsrc/include
CXXFLAGS  := -O3 -std=c++17 -fPIC -fopenmp -Wall -Wextra -Wno-unused-parameter $(INC) -I$(ROCM)/include -D__HIP_PLATFORM_AMD__
HIPFLAGS  := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) $(INC) -Wno-unused-result
MPIFLAGS  := -I$(MPI_HOME)/include
LDROCM    := -L$(ROCM)/lib -lamdhip64 -Wl,-rpath,$(ROCM)/lib
GPU_PLUGIN := mpi_openmp_cuda_amd/lib/libmoc_final_gpu.so

# host core without any ROCm dependency (parser, CPU engine, partitioner, runtime utilities)
CPU_SRCS  := csrc/src/cpu_engine.cpp csrc/src/device_batch.cpp csrc/src/io.cpp csrc/src/partition.cpp csrc/src/problem.cpp csrc/src/wire.cpp \
             csrc/src/score_table.cpp csrc/src/runtime/runtime.cpp csrc/src/runtime/host_region.cpp \
             csrc/src/runtime/kfd_topology.cpp csrc/src/runtime/watchdog.cpp
# host code of the GPU engine (HIP runtime API) and the C ABI of libmoc.so
GPU_SRCS  := csrc/src/hip_engine.cpp csrc/src/capi.cpp csrc/src/runtime/device.cpp csrc/src/runtime/pinned.cpp
CORE_SRCS := $(CPU_SRCS) $(GPU_SRCS)
HIP_SRCS  := $(wildcard csrc/src/hip/*.hip)
CPU_OBJS  := $(patsubst csrc/src/%.cpp,$(OBJ)/%.o,$(CPU_SRCS))
CORE_OBJS := $(patsubst csrc/src/%.cpp,$(OBJ)/%.o,$(CORE_SRCS))
HIP_OBJS  := $(patsubst csrc/src/%.hip,$(OBJ)/%.o,$(HIP_SRCS))
# swipe kernel instances: one code object per (letter form, offsets per lane), from one source
# (csrc/src/hip/swipe_group.inc) — HIP loads only the objects whose kernels a job launches
SWIPE_GROUP := csrc/src/hip/swipe_group.inc
SWIPE_NOFFS := 4 8 12 16 20 24 28 32 36 40 44 48 52 56 60 64
SWIPE_OBJS  := $(foreach lf,0 2,$(foreach no,$(SWIPE_NOFFS),$(OBJ)/hip/swipe_lf$(lf)_n$(no).o))
COMM_OBJS := $(OBJ)/comm/comm.o $(OBJ)/comm/mpi_device_comm.o
RCCL_OBJS := $(OBJ)/comm/rccl_comm.o
HEADERS   := $(shell find csrc/include -name '*.h' -o -name '*.hpp')

.PHONY: all build lib clean run runOn2 test unit asan tsan debug-kernels

all: build
build: lib final $(GPU_PLUGIN)

lib: $(PKG_LIB)

$(OBJ)/%.o: csrc/src/%.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) $(if $(findstring /comm/,$@),$(MPIFLAGS)) -c $< -o $@

$(OBJ)/%.o: csrc/src/%.hip $(HEADERS) $(wildcard csrc/src/hip/*.hpp)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJ)/hip/swipe_lf0_n%.o: $(SWIPE_GROUP) $(HEADERS) $(wildcard csrc/src/hip/*.hpp)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -DMOC_SWIPE_LF=0 -DMOC_SWIPE_NO=$* -x hip -c $< -o $@

$(OBJ)/hip/swipe_lf2_n%.o: $(SWIPE_GROUP) $(HEADERS) $(wildcard csrc/src/hip/*.hpp)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -DMOC_SWIPE_LF=2 -DMOC_SWIPE_NO=$* -x hip -c $< -o $@

$(PKG_LIB): $(CORE_OBJS) $(HIP_OBJS) $(SWIPE_OBJS)
	@mkdir -p $(dir $@)
	$(CXX) -shared -fopenmp -o $@ $^ $(LDROCM) -ldl

# MPICH's conda wrapper names a compiler that is not installed, so link libmpi directly through a
# private directory (keeps /opt/conda/lib — and its older libstdc++ — off the binary's search path).
$(MPILIB)/libmpi.so:
	@mkdir -p $(MPILIB)
	ln -sf $(MPI_HOME)/lib/libmpi.so.12 $(MPILIB)/libmpi.so.12
	ln -sf $(MPI_HOME)/lib/libmpi.so.12 $(MPILIB)/libmpi.so
	ln -sf $(MPI_HOME)/lib/libgfortran.so.4 $(MPILIB)/libgfortran.so.4
	ln -sf $(MPI_HOME)/lib/libquadmath.so.0 $(MPILIB)/libquadmath.so.0

# Build identity baked into ./final (--help, --timing): a hash of the native sources (every file under
# csrc/ plus this Makefile, in sorted order — tests/test_cli.py recomputes it, so a stale prebuilt binary
# shipped next to newer sources is caught even where no .git exists) and the git commit when known.
# The stamp file changes only when the identity does, so an unchanged tree does not relink.
SRC_FILES := $(sort $(wildcard csrc/* csrc/*/* csrc/*/*/* csrc/*/*/*/* csrc/*/*/*/*/*) Makefile)
SRC_HASH  := $(shell cat $(SRC_FILES) 2>/dev/null | sha1sum | cut -c1-12)
GIT_HASH  := $(shell git rev-parse --short=12 HEAD 2>/dev/null || echo unknown)
BUILD_ID  := $(BUILD)/build_id
$(shell mkdir -p $(BUILD); echo 'src=$(SRC_HASH) git=$(GIT_HASH)' | cmp -s - $(BUILD_ID) || echo 'src=$(SRC_HASH) git=$(GIT_HASH)' > $(BUILD_ID))

$(OBJ)/hip/build_info.o: csrc/src/hip/build_info.hip $(BUILD_ID)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -DMOC_SRC_HASH='"$(SRC_HASH)"' -c $< -o $@

$(OBJ)/apps/final.o: csrc/apps/final.cpp csrc/apps/job.hpp $(HEADERS) $(BUILD_ID)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) $(MPIFLAGS) -DMOC_BUILD_ID='"src=$(SRC_HASH) git=$(GIT_HASH)"' -c $< -o $@

$(OBJ)/apps/%.o: csrc/apps/%.cpp csrc/apps/job.hpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) $(MPIFLAGS) -c $< -o $@

# ./final links MPI and the CPU core only; the GPU side is a plugin it dlopens when a rank uses a GPU
APP_OBJS  := $(OBJ)/apps/final.o $(OBJ)/apps/job_common.o $(OBJ)/apps/flow_sliced.o $(OBJ)/apps/flow_stream.o \
             $(OBJ)/apps/text_cut.o $(OBJ)/apps/flow_device_stream.o $(OBJ)/apps/flow_batch.o
final: $(APP_OBJS) $(COMM_OBJS) $(CPU_OBJS) $(MPILIB)/libmpi.so
	$(CXX) -fopenmp -o $@ $(APP_OBJS) $(COMM_OBJS) $(CPU_OBJS) \
	    -L$(MPILIB) -lmpi -Wl,-rpath-link,$(MPI_HOME)/lib -Wl,-rpath,'$$ORIGIN/$(MPILIB)' -ldl

$(GPU_PLUGIN): $(OBJ)/apps/final_gpu.o $(RCCL_OBJS) $(COMM_OBJS) $(PKG_LIB) $(MPILIB)/libmpi.so
	$(CXX) -shared -fopenmp -o $@ $(OBJ)/apps/final_gpu.o $(RCCL_OBJS) $(COMM_OBJS) \
	    -L$(dir $(PKG_LIB)) -lmoc -Wl,-rpath,'$$ORIGIN' -L$(MPILIB) -lmpi -Wl,-rpath-link,$(MPI_HOME)/lib \
	    -Wl,-rpath,'$$ORIGIN/../../$(MPILIB)' $(LDROCM) -lrccl

# Host-side sanitizers (GPU ASan is not available on the target pool). ./final links no ROCm code, so
# the sanitized binaries cover everything the CPU backend runs; a GPU rank would dlopen the plugin.
SAN_SRCS := $(CPU_SRCS) csrc/src/comm/comm.cpp csrc/src/comm/mpi_device_comm.cpp csrc/apps/final.cpp \
            csrc/apps/job_common.cpp csrc/apps/flow_sliced.cpp csrc/apps/flow_stream.cpp csrc/apps/text_cut.cpp \
            csrc/apps/flow_device_stream.cpp csrc/apps/flow_batch.cpp
asan: $(MPILIB)/libmpi.so
	@rm -rf $(BUILD)/asan && mkdir -p $(BUILD)/asan
	for f in $(SAN_SRCS); do \
	  $(CXX) -O1 -g -std=c++17 -fopenmp -fsanitize=address,undefined -fno-omit-frame-pointer $(INC) \
	    -I$(ROCM)/include -D__HIP_PLATFORM_AMD__ $(MPIFLAGS) -c $$f -o $(BUILD)/asan/$$(echo $$f | tr / _).o || exit 1; \
	done
	$(CXX) -fopenmp -fsanitize=address,undefined -o final_asan $(BUILD)/asan/*.o \
	    -L$(MPILIB) -lmpi -Wl,-rpath-link,$(MPI_HOME)/lib -Wl,-rpath,'$$ORIGIN/$(MPILIB)' -ldl

# ThreadSanitizer build of the host paths (OpenMP parser / CPU engine / formatter) — CPU backend only.
# Built with ROCm's clang + LLVM libomp so the Archer OMPT tool (libarcher) can tell TSan about OpenMP
# barriers/tasks; libgomp is not TSan-aware and every parallel-region join reads as a race.
#   make tsan && OMP_TOOL_LIBRARIES=$(ROCM)/lib/llvm/lib/libarcher.so mpiexec -np 2 ./final_tsan --backend=cpu < in
TSAN_CXX  := $(ROCM)/lib/llvm/bin/clang++
tsan: $(MPILIB)/libmpi.so
	@rm -rf $(BUILD)/tsan && mkdir -p $(BUILD)/tsan
	for f in $(SAN_SRCS); do \
	  $(TSAN_CXX) -O1 -g -std=c++17 -fopenmp -fsanitize=thread $(INC) \
	    -I$(ROCM)/include -D__HIP_PLATFORM_AMD__ $(MPIFLAGS) -c $$f -o $(BUILD)/tsan/$$(echo $$f | tr / _).o || exit 1; \
	done
	$(TSAN_CXX) -fopenmp -fsanitize=thread -o final_tsan $(BUILD)/tsan/*.o \
	    -L$(MPILIB) -lmpi -Wl,-rpath-link,$(MPI_HOME)/lib -Wl,-rpath,'$$ORIGIN/$(MPILIB)' \
	    -L$(ROCM)/lib/llvm/lib -Wl,-rpath,$(ROCM)/lib/llvm/lib -ldl

# Device-side bounds checks (MOC_DCHECK: printf, never a fault) in every kernel -> build/debug/libmoc.so;
# select it with MOC_LIB_PATH=$$PWD/build/debug/libmoc.so.
DEBUG_OBJS := $(patsubst csrc/src/hip/%.hip,$(BUILD)/debug/%.hip.o,$(HIP_SRCS)) \
              $(foreach lf,0 2,$(foreach no,$(SWIPE_NOFFS),$(BUILD)/debug/swipe_lf$(lf)_n$(no).hip.o))
debug-kernels: $(BUILD)/debug/libmoc.so
$(BUILD)/debug/libmoc.so: $(CORE_OBJS) $(DEBUG_OBJS)
	$(CXX) -shared -fopenmp -o $@ $^ $(LDROCM) -ldl
$(BUILD)/debug/%.hip.o: csrc/src/hip/%.hip $(HEADERS) $(wildcard csrc/src/hip/*.hpp)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -DMOC_DEBUG_KERNELS -DMOC_SRC_HASH='"$(SRC_HASH)"' -c $< -o $@
$(BUILD)/debug/swipe_lf0_n%.hip.o: $(SWIPE_GROUP) $(HEADERS) $(wildcard csrc/src/hip/*.hpp)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -DMOC_DEBUG_KERNELS -DMOC_SWIPE_LF=0 -DMOC_SWIPE_NO=$* -x hip -c $< -o $@
$(BUILD)/debug/swipe_lf2_n%.hip.o: $(SWIPE_GROUP) $(HEADERS) $(wildcard csrc/src/hip/*.hpp)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -DMOC_DEBUG_KERNELS -DMOC_SWIPE_LF=2 -DMOC_SWIPE_NO=$* -x hip -c $< -o $@

# Kernel A/B builds: make variant NAME=p4 VDEFS="-DMOC_T16_UNROLL=32" -> build/variant_p4/libmoc.so
# (select with MOC_LIB_PATH and MOC_ALLOW_VARIANT_LIB=1: the loader refuses a library whose kernels carry
# defines otherwise; moc_build_info reports them). No switch that gives wrong results lives in the kernel
# sources: a timing-only experiment is a throwaway patch, not a define.
variant: lib
	@mkdir -p $(BUILD)/variant_$(NAME)
	for f in $(HIP_SRCS); do \
	  $(HIPCC) $(HIPFLAGS) $(VDEFS) -DMOC_SRC_HASH='"$(SRC_HASH)"' -DMOC_KERNEL_DEFS='"$(strip $(VDEFS))"' \
	    -c $$f -o $(BUILD)/variant_$(NAME)/$$(basename $$f .hip).hip.o || exit 1; \
	done
	for lf in 0 2; do for no in $(SWIPE_NOFFS); do \
	  $(HIPCC) $(HIPFLAGS) $(VDEFS) -DMOC_SWIPE_LF=$$lf -DMOC_SWIPE_NO=$$no -x hip -c $(SWIPE_GROUP) \
	    -o $(BUILD)/variant_$(NAME)/swipe_lf$${lf}_n$${no}.hip.o || exit 1; \
	done; done
	$(CXX) -shared -fopenmp -o $(BUILD)/variant_$(NAME)/libmoc.so $(CORE_OBJS) $(BUILD)/variant_$(NAME)/*.hip.o $(LDROCM) -ldl

clean:
	rm -rf $(BUILD) final final_asan final_tsan $(PKG_LIB) $(GPU_PLUGIN)

run: build
	$(MPI_HOME)/bin/mpiexec -np $(NP) ./final < $(INPUT)

runOn2: build
	$(MPI_HOME)/bin/mpiexec -np 2 -machinefile mf --map-by node ./final < $(INPUT)

test: unit
	python -m pytest tests/ -x -q -m "not gpu"

# native unit tests of the host core (no GPU, no MPI)
$(BUILD)/test_core: csrc/tests/test_core.cpp csrc/apps/text_cut.cpp csrc/apps/text_cut.hpp $(CPU_OBJS) $(HEADERS)
	$(CXX) $(CXXFLAGS) -o $@ csrc/tests/test_core.cpp csrc/apps/text_cut.cpp $(CPU_OBJS) -ldl

unit: $(BUILD)/test_core
	$(BUILD)/test_core

# parser throughput (count vs fill, SIMD A/B): build/fill_bench [records]
$(BUILD)/fill_bench: tools/fill_bench.cpp $(CPU_OBJS) $(HEADERS)
	$(CXX) $(CXXFLAGS) -o $@ tools/fill_bench.cpp $(CPU_OBJS) -ldl
