# Build for the SDA MI355X framework.
#
#   make            -> host core library, pybind11 modules, CLI binaries, HIP module
#   make host       -> everything except the HIP (gfx950) extension
#   make asan       -> AddressSanitizer/UBSan build of the host test binary
#
# Outputs (in-tree, git-ignored, shipped to the GPU box with the snapshot):
#   sda_amd/_lib/_sda_native<EXT>   host control plane + crypto bindings
#   sda_amd/_lib/_sda_gpu<EXT>      HIP/CDNA4 kernels (hipcc --offload-arch=gfx950)
#   sda_amd/_lib/libsda_device.so   the client roles' GPU backend (kernels + C++ driver),
#                                   loaded on demand by `sda --device gpu` and the Python client
#   sda_amd/_lib/bin/sda, sdad      agent CLI and server daemon

PYTHON   ?= python3
CXX      ?= g++
ROCM     ?= /opt/rocm
HIPCC    ?= $(ROCM)/bin/hipcc
GPU_ARCH ?= gfx950

EXT        := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
PY_INC     := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_paths()['include'])")
PYBIND_INC := $(shell $(PYTHON) -c "import pybind11;print(pybind11.get_include())")

BUILD := build
LIB   := sda_amd/_lib
BIN   := $(LIB)/bin

CXXFLAGS ?= -O3 -g -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter -pthread
INCS     := -Icsrc/include
# packed-fp32 VALU forms are switched off for every device compile (the host
# pass warns that it does not know the feature; harmless)
NO_PK_F32 := -Xclang -target-feature -Xclang -packed-fp32-ops
HIPFLAGS := -O3 -std=c++17 -fPIC --offload-arch=$(GPU_ARCH) -Wall -Wno-unused-parameter \
            -Wno-unused-result -munsafe-fp-atomics $(NO_PK_F32)

CORE_SRC := $(wildcard csrc/src/*.cc)
CORE_OBJ := $(patsubst csrc/src/%.cc,$(BUILD)/core/%.o,$(CORE_SRC))
CORE_LIB := $(BUILD)/libsdacore.a

PY_SRC   := $(wildcard csrc/python/*.cc)
PY_OBJ   := $(patsubst csrc/python/%.cc,$(BUILD)/py/%.o,$(PY_SRC))

HIP_SRC  := $(wildcard csrc/kernels/*.hip)
HIP_OBJ  := $(patsubst csrc/kernels/%.hip,$(BUILD)/hip/%.o,$(HIP_SRC))
HIP_BIND := csrc/kernels/gpu_module.cpp

NATIVE_MOD := $(LIB)/_sda_native$(EXT)
GPU_MOD    := $(LIB)/_sda_gpu$(EXT)
DEVICE_LIB := $(LIB)/libsda_device.so
BINS       := $(patsubst csrc/bin/%.cc,$(BIN)/%,$(wildcard csrc/bin/*.cc))

.PHONY: all host gpu clean asan tsan selftest emul check
all: host gpu
host: $(NATIVE_MOD) $(BINS)
gpu: $(GPU_MOD) $(DEVICE_LIB)

$(BUILD)/core/%.o: csrc/src/%.cc $(wildcard csrc/include/sda/*.hpp)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) $(INCS) -c $< -o $@

$(CORE_LIB): $(CORE_OBJ)
	@mkdir -p $(dir $@)
	rm -f $@ && ar rcs $@ $^

$(BUILD)/py/%.o: csrc/python/%.cc $(wildcard csrc/include/sda/*.hpp)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -fvisibility=hidden $(INCS) -I$(PY_INC) -I$(PYBIND_INC) -c $< -o $@

$(NATIVE_MOD): $(PY_OBJ) $(CORE_LIB)
	@mkdir -p $(dir $@)
	$(CXX) -shared -o $@ $(PY_OBJ) $(CORE_LIB) -pthread -ldl

$(BIN)/%: csrc/bin/%.cc $(CORE_LIB)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) $(INCS) $< $(CORE_LIB) -o $@ -pthread -ldl

$(BUILD)/hip/%.o: csrc/kernels/%.hip $(wildcard csrc/kernels/*.hpp) $(wildcard csrc/kernels/*.inc) $(wildcard csrc/include/sda/*.hpp)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) $(INCS) -c $< -o $@

$(BUILD)/hip/gpu_module.o: $(HIP_BIND) $(wildcard csrc/kernels/*.hpp) $(wildcard csrc/include/sda/*.hpp)
	@mkdir -p $(dir $@)
	$(HIPCC) -O3 -std=c++17 -fPIC -fvisibility=hidden $(INCS) -I$(PY_INC) -I$(PYBIND_INC) -c $< -o $@

$(GPU_MOD): $(HIP_OBJ) $(BUILD)/hip/gpu_module.o $(CORE_LIB)
	@mkdir -p $(dir $@)
	$(HIPCC) -shared --offload-arch=$(GPU_ARCH) -o $@ $^ -pthread -ldl

# the roles' GPU backend: host C++ driving the same kernel objects
$(BUILD)/hip/device_backend.o: csrc/device/device_backend.cc $(wildcard csrc/kernels/*.hpp) $(wildcard csrc/include/sda/*.hpp)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -Wno-unused-result -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include $(INCS) -c $< -o $@

$(DEVICE_LIB): $(HIP_OBJ) $(BUILD)/hip/device_backend.o $(CORE_LIB)
	@mkdir -p $(dir $@)
	$(HIPCC) -shared --offload-arch=$(GPU_ARCH) -o $@ $^ -pthread -ldl

# sanitizer builds of the host control plane; run the C++ self-test
asan: $(BUILD)/asan/sda_selftest
	$(BUILD)/asan/sda_selftest
$(BUILD)/asan/sda_selftest: csrc/bin/sda_selftest.cc $(CORE_SRC) $(wildcard csrc/include/sda/*.hpp)
	@mkdir -p $(BUILD)/asan
	$(CXX) -O1 -g -std=c++17 -fsanitize=address,undefined -fno-sanitize-recover=undefined \
	    -fno-omit-frame-pointer $(INCS) csrc/bin/sda_selftest.cc $(CORE_SRC) \
	    -o $@ -pthread -ldl
tsan: $(BUILD)/tsan/sda_selftest
	TSAN_OPTIONS=halt_on_error=1 $(BUILD)/tsan/sda_selftest
$(BUILD)/tsan/sda_selftest: csrc/bin/sda_selftest.cc $(CORE_SRC) $(wildcard csrc/include/sda/*.hpp)
	@mkdir -p $(BUILD)/tsan
	$(CXX) -O1 -g -std=c++17 -fsanitize=thread -fno-omit-frame-pointer $(INCS) \
	    csrc/bin/sda_selftest.cc $(CORE_SRC) -o $@ -pthread -ldl
selftest: $(BIN)/sda_selftest
	$(BIN)/sda_selftest

clean:
	rm -rf $(BUILD) $(LIB)/*.so $(BIN)

# one command for everything a checkout must pass without a GPU: build, the CPU test
# suite (protocol, stores, REST, CLI walkthrough with an asserted output, crypto
# KATs, gloo multi-process rounds), the sanitizer self-tests and the host emulation
# of the device algorithms
check: all
	$(PYTHON) -m pytest tests -x -q -m "not gpu"
	$(MAKE) asan tsan emul
	bash docs/cli-walkthrough.sh > /dev/null

# host emulation of the device algorithms (no GPU needed)
emul: $(BUILD)/hip/host_emul
	$(BUILD)/hip/host_emul
$(BUILD)/hip/host_emul: csrc/kernels/host_emul.cpp $(wildcard csrc/kernels/*.hpp) csrc/kernels/ed25519_base.inc $(CORE_LIB)
	@mkdir -p $(dir $@)
	$(HIPCC) -O2 -std=c++17 --offload-arch=$(GPU_ARCH) $(NO_PK_F32) $(INCS) -c $< -o $@.o
	$(HIPCC) --offload-arch=$(GPU_ARCH) $@.o $(CORE_LIB) -o $@ -pthread -ldl
