# libstereo_hip.so — gfx950 HIP kernels behind the C ABI in include/stereo_hip.h
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
PKG      := stereo_depth_estimation_amd
SRCS     := $(wildcard $(PKG)/csrc/*.hip)
CPPSRCS  := $(wildcard $(PKG)/csrc/*.cpp)
OBJS     := $(patsubst $(PKG)/csrc/%.hip,build/%.o,$(SRCS)) $(patsubst $(PKG)/csrc/%.cpp,build/%.cpp.o,$(CPPSRCS))
LIB      := $(PKG)/libstereo_hip.so
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Iinclude

all: $(LIB)

build/%.o: $(PKG)/csrc/%.hip $(PKG)/csrc/common.h $(PKG)/csrc/halo_util.h include/stereo_hip.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# host-only C++ (the cache reader): no device code
build/%.cpp.o: $(PKG)/csrc/%.cpp include/stereo_hip.h
	@mkdir -p build
	$(CXX) -O3 -std=c++17 -fPIC -Wall -pthread -Iinclude -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -pthread -o $@ $(OBJS) -lz

clean:
	rm -rf build $(LIB)

.PHONY: all clean
