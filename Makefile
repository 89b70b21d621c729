# Build everything in-tree (the .so files travel to the GPU box with the snapshot).
#   make            -> subspace_amd/libsubspace_crc.so (gfx950 HIP + host C++) and oracle/liboracle_crc.so
#   make test-cpu   -> CPU test suite
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result
CSRC := subspace_amd/csrc
LIB := subspace_amd/libsubspace_crc.so
OBJDIR := build/obj

HIP_SRCS := $(CSRC)/crc_uniform.hip $(CSRC)/crc_ragged.hip $(CSRC)/crc_long.hip $(CSRC)/crc_combine.hip $(CSRC)/crc_slots.hip $(CSRC)/capi.hip $(CSRC)/testutil.hip
CPP_SRCS := $(CSRC)/host_crc.cpp
HDRS := $(CSRC)/crc_device.h $(CSRC)/crc_math.h include/subspace_crc.h
OBJS := $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.o,$(HIP_SRCS)) $(patsubst $(CSRC)/%.cpp,$(OBJDIR)/%.o,$(CPP_SRCS))

all: $(LIB) oracle tools/config_a tools/drain_demo

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	g++ -O3 -std=c++17 -fPIC -Wall -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

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

test-cpu: all
	python -m pytest tests/ -x -q -m "not gpu"

clean:
	rm -rf build $(LIB) tools/config_a tools/drain_demo
	$(MAKE) -C oracle clean

.PHONY: all oracle test-cpu clean
