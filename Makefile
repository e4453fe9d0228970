# Builds libtmr.so (gfx950) in-tree.  `python __graft_entry__.py build` drives this too.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
SRC := $(wildcard tmrnet_amd/csrc/*.hip) tmrnet_amd/csrc/api.cpp
OBJ := $(patsubst tmrnet_amd/csrc/%,build/%.o,$(SRC))
CFLAGS := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Iinclude -Itmrnet_amd/csrc -munsafe-fp-atomics

tmrnet_amd/libtmr.so: $(OBJ)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(OBJ)

build/%.hip.o: tmrnet_amd/csrc/%.hip tmrnet_amd/csrc/common.h tmrnet_amd/csrc/gemm_kernel.h tmrnet_amd/csrc/gemm16_kernel.h include/tmr.h
	@mkdir -p build
	$(HIPCC) $(CFLAGS) -c $< -o $@

build/%.cpp.o: tmrnet_amd/csrc/%.cpp tmrnet_amd/csrc/common.h include/tmr.h
	@mkdir -p build
	$(HIPCC) $(CFLAGS) -c $< -o $@

clean:
	rm -rf build tmrnet_amd/libtmr.so
.PHONY: clean
