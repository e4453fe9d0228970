# Builds libtmr.so (gfx950) in-tree.  `python __graft_entry__.py build` drives this too.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
SRC := $(wildcard tmrnet_amd/csrc/*.hip) tmrnet_amd/csrc/api.cpp
OBJ := $(patsubst tmrnet_amd/csrc/%,build/%.o,$(SRC))
CFLAGS := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Iinclude -Itmrnet_amd/csrc -munsafe-fp-atomics

tmrnet_amd/libtmr.so: $(OBJ)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(OBJ)

# header dependencies from the compiler (-MMD: build/*.d); an edit of the LDS-DMA engine
# (gemm16_kernel.h) rebuilds only the gemm16_<view>_<prec>.hip units
build/%.hip.o: tmrnet_amd/csrc/%.hip
	@mkdir -p build
	$(HIPCC) $(CFLAGS) -MMD -MP -c $< -o $@

build/%.cpp.o: tmrnet_amd/csrc/%.cpp
	@mkdir -p build
	$(HIPCC) $(CFLAGS) -MMD -MP -c $< -o $@

-include $(OBJ:.o=.d)

clean:
	rm -rf build tmrnet_amd/libtmr.so
.PHONY: clean
