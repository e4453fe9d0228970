# Builds libtmr.so (gfx950) in-tree.  `python __graft_entry__.py build` drives this too.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
# PROLOGUES=1: the A/B build with the retired operand prologues (include/tmr_prologue.h) compiled
# in and exported, as tmrnet_amd/libtmr_pro.so from objects under build_pro/ (the default
# libtmr.so never carries them)
PROLOGUES ?= 0
ifeq ($(PROLOGUES),1)
BUILD := build_pro
LIB := tmrnet_amd/libtmr_pro.so
else
BUILD := build
LIB := tmrnet_amd/libtmr.so
endif
SRC := $(wildcard tmrnet_amd/csrc/*.hip) tmrnet_amd/csrc/api.cpp
OBJ := $(patsubst tmrnet_amd/csrc/%,$(BUILD)/%.o,$(SRC))
CFLAGS := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Iinclude -Itmrnet_amd/csrc -munsafe-fp-atomics \
          -DTMR_PROLOGUES=$(PROLOGUES) $(EXTRA)

$(LIB): $(OBJ)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(OBJ)

# header dependencies from the compiler (-MMD: build/*.d); an edit of the LDS-DMA engine
# (gemm16_kernel.h) rebuilds only the gemm16_<view>_<prec>.hip units
$(BUILD)/%.hip.o: tmrnet_amd/csrc/%.hip
	@mkdir -p $(BUILD)
	$(HIPCC) $(CFLAGS) -MMD -MP -c $< -o $@

$(BUILD)/%.cpp.o: tmrnet_amd/csrc/%.cpp
	@mkdir -p $(BUILD)
	$(HIPCC) $(CFLAGS) -MMD -MP -c $< -o $@

-include $(OBJ:.o=.d)

clean:
	rm -rf build build_pro tmrnet_amd/libtmr.so tmrnet_amd/libtmr_pro.so
.PHONY: clean
