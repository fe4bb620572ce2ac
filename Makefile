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
HIPFLAGS  := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Iinclude

HOST_SRC  := $(CSRC)/host/storage.cpp $(CSRC)/host/device.cpp $(CSRC)/host/operators.cpp $(CSRC)/host/aggregate.cpp \
             $(CSRC)/host/projection.cpp $(CSRC)/host/binary_io.cpp $(CSRC)/host/scheduler.cpp
HOST_HDR  := $(wildcard $(CSRC)/host/*.hpp) include/hyrise_amd.h include/hyrise_amd_trace.h

all: $(LIB)/libhyrise_amd.so $(LIB)/libhyrise_host.so $(LIB)/_hyrise_host$(EXTSUF) $(LIB)/exchange_check $(LIB)/host_concurrency_check_tsan

# host-side concurrency checks (deferred tables, job groups, chunk reaper) under ThreadSanitizer: no GPU, run by
# tests/test_host_concurrency.py
$(LIB)/host_concurrency_check_tsan: tests/native/host_concurrency_check.cpp $(CSRC)/host/storage.cpp $(CSRC)/host/scheduler.cpp $(HOST_HDR)
	@mkdir -p $(LIB)
	$(CXX) -std=c++17 -O1 -g -fsanitize=thread -I$(CSRC)/host -Iinclude -o $@ $< $(CSRC)/host/storage.cpp $(CSRC)/host/scheduler.cpp -lpthread

# native (no Python, no torch) check of the C-ABI RCCL exchange, run by tests/test_dist_join_gpu.py on the GPU
$(LIB)/exchange_check: tests/native/exchange_check.cpp include/hyrise_amd.h $(LIB)/libhyrise_amd.so
	$(HIPCC) -std=c++17 -O2 -Iinclude -o $@ $< -L$(LIB) -lhyrise_amd -Wl,-rpath,'$$ORIGIN'

CAPI_HDR  := include/hyrise_amd.h $(CSRC)/capi/capi_common.hpp $(CSRC)/kernels/common.hpp

# one object per C-ABI translation unit (they compile in parallel under make -j)
$(LIB)/hyrise_amd.o: $(CSRC)/capi/hyrise_amd.hip $(CSRC)/kernels/scan.hip $(CSRC)/kernels/join.hip $(CAPI_HDR)
	@mkdir -p $(LIB)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIB)/hyrise_amd_aggregate.o: $(CSRC)/capi/hyrise_amd_aggregate.hip $(CSRC)/kernels/aggregate.hip $(CSRC)/kernels/projection.hip \
                                $(CSRC)/kernels/aggregate_fused.hip $(CSRC)/kernels/aggregate_lanes.hip \
                                $(CSRC)/kernels/aggregate_vec.hip $(CSRC)/kernels/aggregate_stream.hip $(CAPI_HDR) \
                                $(CSRC)/capi/agg_jit.hpp $(CSRC)/kernels/agg_jit_prelude.hpp
	@mkdir -p $(LIB)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

JOIN_TUS   := join join_i32 join_i64 join_f32 join_f64
JOIN_OBJS  := $(patsubst %,$(LIB)/hyrise_amd_%.o,$(JOIN_TUS))

$(JOIN_OBJS): $(LIB)/hyrise_amd_%.o: $(CSRC)/capi/hyrise_amd_%.hip $(CSRC)/capi/join_host.hpp $(CSRC)/kernels/join.hip $(CSRC)/kernels/join_direct.hip $(CAPI_HDR)
	@mkdir -p $(LIB)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

# plan-compiled aggregation: host code (hiprtc) with the device prelude embedded as text
$(LIB)/agg_jit_prelude.inc: $(CSRC)/kernels/agg_jit_prelude.hpp tools/embed_text.py
	@mkdir -p $(LIB)
	$(PY) tools/embed_text.py kJitPrelude $< > $@

$(LIB)/hyrise_amd_agg_jit.o: $(CSRC)/capi/hyrise_amd_agg_jit.cpp $(CSRC)/capi/agg_jit.hpp $(CSRC)/kernels/agg_jit_prelude.hpp \
                             $(LIB)/agg_jit_prelude.inc include/hyrise_amd.h
	$(HIPCC) --offload-arch=$(ARCH) -std=c++17 -O2 -fPIC -Iinclude -I$(LIB) -c -o $@ $<

$(LIB)/hyrise_amd_order.o: $(CSRC)/capi/hyrise_amd_order.hip $(CAPI_HDR)
	@mkdir -p $(LIB)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIB)/hyrise_amd_comm.o: $(CSRC)/capi/hyrise_amd_comm.hip $(CAPI_HDR)
	@mkdir -p $(LIB)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIB)/hyrise_amd_compare.o: $(CSRC)/capi/hyrise_amd_compare.hip $(CAPI_HDR)
	@mkdir -p $(LIB)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIB)/hyrise_amd_validate.o: $(CSRC)/capi/hyrise_amd_validate.hip $(CAPI_HDR)
	@mkdir -p $(LIB)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIB)/hyrise_amd_decode.o: $(CSRC)/capi/hyrise_amd_decode.hip $(CAPI_HDR)
	@mkdir -p $(LIB)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIB)/hyrise_amd_trace.o: $(CSRC)/capi/hyrise_amd_trace.hip include/hyrise_amd_trace.h $(CSRC)/capi/capi_common.hpp
	@mkdir -p $(LIB)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIB)/hyrise_amd_string.o: $(CSRC)/capi/hyrise_amd_string.hip $(CAPI_HDR)
	@mkdir -p $(LIB)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIB)/libhyrise_amd.so: $(LIB)/hyrise_amd.o $(LIB)/hyrise_amd_aggregate.o $(LIB)/hyrise_amd_order.o \
                         $(LIB)/hyrise_amd_comm.o $(LIB)/hyrise_amd_compare.o \
                         $(LIB)/hyrise_amd_validate.o $(LIB)/hyrise_amd_decode.o $(LIB)/hyrise_amd_string.o \
                         $(LIB)/hyrise_amd_agg_jit.o $(LIB)/hyrise_amd_trace.o $(JOIN_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -L/opt/rocm/lib -lrccl -lhiprtc -Wl,-rpath,/opt/rocm/lib

$(LIB)/libhyrise_host.so: $(HOST_SRC) $(HOST_HDR) $(LIB)/libhyrise_amd.so
	$(CXX) $(CXXFLAGS) -I/opt/rocm/include -shared -o $@ $(HOST_SRC) -L$(LIB) -lhyrise_amd -L/opt/rocm/lib \
	  -lrocprofiler-sdk-roctx -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,/opt/rocm/lib

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
