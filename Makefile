# Build everything in-tree (the .so files travel to the GPU box with the snapshot).
#   make            -> subspace_amd/libsubspace_crc.so (gfx950 HIP + host C++) and oracle/liboracle_crc.so
#   make test-cpu   -> CPU test suite
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result
CSRC := subspace_amd/csrc
LIB := subspace_amd/libsubspace_crc.so
OBJDIR := build/obj

HIP_SRCS := $(CSRC)/crc_uniform.hip $(CSRC)/crc_small.hip $(CSRC)/crc_ragged.hip $(CSRC)/crc_long.hip $(CSRC)/crc_combine.hip $(CSRC)/crc_slots.hip $(CSRC)/capi.hip
CPP_SRCS := $(CSRC)/host_crc.cpp $(CSRC)/split_alloc.cpp
HDRS := $(CSRC)/crc_device.h $(CSRC)/crc_math.h $(CSRC)/ctx.h include/subspace_crc.h
OBJS := $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.o,$(HIP_SRCS)) $(patsubst $(CSRC)/%.cpp,$(OBJDIR)/%.o,$(CPP_SRCS))
# the product library exports exactly the public header's functions (exports.map)
EXPORTS := $(CSRC)/exports.map
# tests / bench / tools only: development knobs, probes, synthetic-payload generators and read
# probes (devtools.hip, testutil.hip); never linked by a client, not needed by the product
DEVLIB := subspace_amd/libsubspace_crc_dev.so
DEV_OBJS := $(OBJDIR)/devtools.o $(OBJDIR)/testutil.o

all: $(LIB) $(DEVLIB) oracle tools/config_a tools/drain_demo tools/batch_gates

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	g++ -O3 -std=c++17 -fPIC -Wall -c $< -o $@

$(LIB): $(OBJS) $(EXPORTS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -Wl,--version-script=$(EXPORTS) -o $@ $(OBJS)

$(OBJDIR)/devtools.o: $(CSRC)/devtools.hip $(CSRC)/crc_small.hip $(CSRC)/crc_uniform.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/testutil.o: $(CSRC)/testutil.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(DEVLIB): $(DEV_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(DEV_OBJS)

oracle:
	$(MAKE) -C oracle

# config A (CPU plumbing: 1 pub x 1 sub calc+verify latency through the drop-in header)
tools/config_a: tools/config_a.cpp include/subspace/checksum.h $(LIB)
	g++ -O2 -std=c++17 -Iinclude -o $@ tools/config_a.cpp -Lsubspace_amd -lsubspace_crc \
	    -Wl,-rpath,'$$ORIGIN/../subspace_amd' -ldl

# subscriber drain / batch publish through the header-only C++ helper (a GPU test runs it)
tools/drain_demo: tools/drain_demo.cpp include/subspace/checksum.h include/subspace/checksum_batch.h include/subspace_crc.h $(LIB)
	g++ -O2 -std=c++17 -Wall -Iinclude -o $@ tools/drain_demo.cpp -Lsubspace_amd -lsubspace_crc \
	    -Wl,-rpath,'$$ORIGIN/../subspace_amd'

# the ValidateChecksum / publisher gates of the C++ helper (tests/test_batch_gates.py)
tools/batch_gates: tests/c/batch_gates.cpp include/subspace/checksum.h include/subspace/checksum_batch.h include/subspace_crc.h $(LIB)
	g++ -O2 -std=c++17 -Wall -Wextra -Iinclude -o $@ tests/c/batch_gates.cpp -Lsubspace_amd -lsubspace_crc \
	    -Wl,-rpath,'$$ORIGIN/../subspace_amd'

test-cpu: all
	python -m pytest tests/ -x -q -m "not gpu"

# ---- AddressSanitizer + UBSan build of the host code (CPU only; GPU sanitizers are not
# available on the pool): the host sources (host CRC, split allocator) AND capi.hip's host
# side (-Xarch_host: argument validation, workspace sizing, the chunked host-slot pipeline,
# the host-address -> device-alias translation, the call scope and stream ordering) are
# instrumented, all with ROCm's clang so one ASan runtime (clang's, shared) serves
# everything; the other HIP objects (kernel launch stubs only) are linked in unchanged.
# python runs with that runtime preloaded, ASan's leak checker off (CPython's own
# allocations), every UBSan finding fatal.
ASAN_DIR := build/asan
ASAN_CXX := /opt/rocm/llvm/bin/clang++
ASAN_CC := /opt/rocm/llvm/bin/clang
ASAN_FLAGS := -fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=all -g -O1 -shared-libsan
ASAN_RT := $(shell $(ASAN_CXX) -print-file-name=libclang_rt.asan-x86_64.so)
ASAN_LIB := $(ASAN_DIR)/libsubspace_crc.so
ASAN_HOST_OBJS := $(patsubst $(CSRC)/%.cpp,$(ASAN_DIR)/%.o,$(CPP_SRCS)) $(ASAN_DIR)/capi.o
HIP_OBJS := $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.o,$(HIP_SRCS))
ASAN_HIP_OBJS := $(filter-out $(OBJDIR)/capi.o,$(HIP_OBJS))

$(ASAN_DIR)/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(ASAN_DIR)
	$(ASAN_CXX) -std=c++17 -fPIC -Wall $(ASAN_FLAGS) -c $< -o $@

$(ASAN_DIR)/capi.o: $(CSRC)/capi.hip $(HDRS)
	@mkdir -p $(ASAN_DIR)
	$(HIPCC) $(HIPFLAGS) -g -Xarch_host -fsanitize=address,undefined -Xarch_host -fno-sanitize-recover=all \
	    -Xarch_host -fno-omit-frame-pointer -c $< -o $@

$(ASAN_LIB): $(ASAN_HOST_OBJS) $(ASAN_HIP_OBJS) $(EXPORTS)
	$(ASAN_CXX) -shared -fPIC $(ASAN_FLAGS) -Wl,--version-script=$(EXPORTS) -o $@ $(ASAN_HOST_OBJS) $(ASAN_HIP_OBJS) -L/opt/rocm/lib -lamdhip64 \
	    -Wl,-rpath,/opt/rocm/lib

$(ASAN_DIR)/config_a: tools/config_a.cpp include/subspace/checksum.h $(ASAN_LIB)
	$(ASAN_CXX) -std=c++17 $(ASAN_FLAGS) -Iinclude -o $@ tools/config_a.cpp -L$(ASAN_DIR) -lsubspace_crc -Wl,-rpath,'$$ORIGIN' -ldl

$(ASAN_DIR)/drain_demo: tools/drain_demo.cpp include/subspace/checksum.h include/subspace/checksum_batch.h include/subspace_crc.h $(ASAN_LIB)
	$(ASAN_CXX) -std=c++17 -Wall $(ASAN_FLAGS) -Iinclude -o $@ tools/drain_demo.cpp -L$(ASAN_DIR) -lsubspace_crc -Wl,-rpath,'$$ORIGIN'

$(ASAN_DIR)/batch_gates: tests/c/batch_gates.cpp include/subspace/checksum.h include/subspace/checksum_batch.h include/subspace_crc.h $(ASAN_LIB)
	$(ASAN_CXX) -std=c++17 -Wall $(ASAN_FLAGS) -Iinclude -o $@ tests/c/batch_gates.cpp -L$(ASAN_DIR) -lsubspace_crc -Wl,-rpath,'$$ORIGIN'

$(ASAN_DIR)/c_binding: tests/c/c_binding.c include/subspace_crc.h $(ASAN_LIB)
	$(ASAN_CC) -std=c11 -Wall -Wextra $(ASAN_FLAGS) -Iinclude -o $@ tests/c/c_binding.c -L$(ASAN_DIR) -lsubspace_crc -Wl,-rpath,'$$ORIGIN'

asan: $(ASAN_LIB) $(ASAN_DIR)/config_a $(ASAN_DIR)/drain_demo $(ASAN_DIR)/c_binding $(ASAN_DIR)/batch_gates

asan-test: asan oracle
	ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
	LD_PRELOAD="$(ASAN_RT)" \
	SUBSPACE_CRC_PROBE_LIB=$(CURDIR)/$(ASAN_LIB) SUBSPACE_CRC_ASAN_DIR=$(CURDIR)/$(ASAN_DIR) \
	python -m pytest tests/test_host_api.py tests/test_capi.py tests/test_split_alloc.py tests/test_c_binding.py tests/test_batch_gates.py -q -m "not gpu" -p no:cacheprovider

# ---- ThreadSanitizer build of the host code: the g++ host sources and capi.hip's host side
# (-Xarch_host) instrumented, compiled and linked with ROCm's clang so one TSan runtime serves
# all; tools/tsan_stress.cpp drives every host entry point from 8 threads at once.
TSAN_DIR := build/tsan
TSAN_CXX := /opt/rocm/llvm/bin/clang++
TSAN_FLAGS := -fsanitize=thread -g -O1
TSAN_LIB := $(TSAN_DIR)/libsubspace_crc.so
TSAN_HOST_OBJS := $(patsubst $(CSRC)/%.cpp,$(TSAN_DIR)/%.o,$(CPP_SRCS)) $(TSAN_DIR)/capi.o
TSAN_HIP_OBJS := $(filter-out $(OBJDIR)/capi.o,$(HIP_OBJS))

$(TSAN_DIR)/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(TSAN_DIR)
	$(TSAN_CXX) -std=c++17 -fPIC -Wall $(TSAN_FLAGS) -c $< -o $@

$(TSAN_DIR)/capi.o: $(CSRC)/capi.hip $(HDRS)
	@mkdir -p $(TSAN_DIR)
	$(HIPCC) $(HIPFLAGS) -g -Xarch_host -fsanitize=thread -c $< -o $@

$(TSAN_LIB): $(TSAN_HOST_OBJS) $(TSAN_HIP_OBJS)
	$(TSAN_CXX) -shared -fPIC -fsanitize=thread -o $@ $(TSAN_HOST_OBJS) $(TSAN_HIP_OBJS) \
	    -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib

$(TSAN_DIR)/tsan_stress: tools/tsan_stress.cpp include/subspace_crc.h include/subspace/checksum.h $(TSAN_LIB)
	$(TSAN_CXX) -std=c++17 -Wall $(TSAN_FLAGS) -Iinclude -o $@ tools/tsan_stress.cpp -L$(TSAN_DIR) -lsubspace_crc \
	    -Wl,-rpath,'$$ORIGIN' -lpthread

tsan: $(TSAN_DIR)/tsan_stress

tsan-test: tsan
	TSAN_OPTIONS=halt_on_error=1:exitcode=66 $(TSAN_DIR)/tsan_stress 8 200

clean:
	rm -rf build $(LIB) $(DEVLIB) tools/config_a tools/drain_demo tools/batch_gates
	$(MAKE) -C oracle clean

.PHONY: all oracle test-cpu clean asan asan-test tsan tsan-test
