# Build of the MI355X (gfx950) execution layer. `make` builds the product libraries in-tree under
# hyrise-1_amd/_lib/; `make oracle` builds the CPU restatement used only by tests/bench baselines;
# `make ref` compiles the reference's own murmur_hash.cpp + tpch-dbgen sources (only where /root/reference exists).
PY        ?= python3
HIPCC     ?= hipcc
CXX       ?= g++
ARCH      ?= gfx950
LIB       := hyrise-1_amd/_lib
CSRC      := hyrise-1_amd/csrc
PYINC     := $(shell $(PY) -c "import sysconfig;print(sysconfig.get_paths()['include'])")
PYBIND    := $(shell $(PY) -c "import pybind11;print(pybind11.get_include())")
EXTSUF    := $(shell $(PY) -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
CXXFLAGS  := -std=c++17 -O2 -fPIC -Wall -Wno-unused-function -Iinclude -I$(CSRC)/host
HIPFLAGS  := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Iinclude

HOST_SRC  := $(CSRC)/host/storage.cpp $(CSRC)/host/device.cpp $(CSRC)/host/operators.cpp
HOST_HDR  := $(wildcard $(CSRC)/host/*.hpp) include/hyrise_amd.h
KERN_SRC  := $(CSRC)/capi/hyrise_amd.hip $(wildcard $(CSRC)/kernels/*.hip) $(wildcard $(CSRC)/kernels/*.hpp)

all: $(LIB)/libhyrise_amd.so $(LIB)/libhyrise_host.so $(LIB)/_hyrise_host$(EXTSUF)

$(LIB)/libhyrise_amd.so: $(KERN_SRC) include/hyrise_amd.h
	@mkdir -p $(LIB)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(CSRC)/capi/hyrise_amd.hip

$(LIB)/libhyrise_host.so: $(HOST_SRC) $(HOST_HDR) $(LIB)/libhyrise_amd.so
	$(CXX) $(CXXFLAGS) -shared -o $@ $(HOST_SRC) -L$(LIB) -lhyrise_amd -Wl,-rpath,'$$ORIGIN'

$(LIB)/_hyrise_host$(EXTSUF): $(CSRC)/host/bindings.cpp $(HOST_HDR) $(LIB)/libhyrise_host.so
	$(CXX) $(CXXFLAGS) -I$(PYINC) -I$(PYBIND) -shared -o $@ $(CSRC)/host/bindings.cpp -L$(LIB) -lhyrise_host \
	  -lhyrise_amd -Wl,-rpath,'$$ORIGIN'

oracle: all
	$(MAKE) -C oracle

ref:
	$(MAKE) -C oracle ref

clean:
	rm -rf $(LIB) oracle/_build

.PHONY: all oracle ref clean
