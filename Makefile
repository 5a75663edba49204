# Build of the MI355X IPv4 fast path (gfx950) and of the test oracle.
# Everything is built in-tree so the shared objects travel to the GPU box.
HIPCC ?= /opt/rocm/bin/hipcc
CC ?= gcc
ARCH ?= gfx950
# host code built here runs on the GPU box's host too: portable x86-64-v3
CFLAGS_HOST = -O3 -march=x86-64-v3 -fPIC -Wall -Wextra -Wno-unused-parameter
HIPFLAGS = -x hip --offload-arch=$(ARCH) -O3 -fPIC -Wall -Wno-unused-value -Wno-unused-result -std=c++17 $(EXTRA_HIPFLAGS)

CSRC = grout_amd/csrc
BUILD = build
LIB_HIP = grout_amd/libgrout_hip.so
LIB_HOST = grout_amd/libgrout_host.so
LIB_ORACLE = oracle/liboracle.so
# The grout module (what grout builds in modules/gpu):
# the node, the control-plane mirror, the CPU continuation nodes. It includes
# grout's and DPDK's headers by name; here the include path leads those names
# to the test stand-ins, and the library leaves grout's / DPDK's symbols
# undefined (the stand-in library that loads it provides them).
MOD = grout_amd/module
LIB_MOD = grout_amd/libgrout_gpu_fwd4.so
MOD_SRC = $(MOD)/gpu_fwd4_node.c $(MOD)/gpu_fwd4_control.c $(MOD)/gpu_fwd4_cpu_nodes.c
MOD_HDRS = $(MOD)/gpu_fwd4_node.h $(MOD)/gpu_fwd4_control.h include/grout_hip.h
# Test infrastructure: the rte_graph / grout stand-ins and the walk and
# control harnesses, linked against the module library.
STANDIN = tests/standin
LIB_STANDIN = $(STANDIN)/libgrout_standin.so
STANDIN_SRC = $(STANDIN)/rte_graph_min.c $(STANDIN)/rte_rcu_min.c $(STANDIN)/gr_datapath_min.c \
	$(STANDIN)/gr_control_min.c $(STANDIN)/walk_harness.c $(STANDIN)/control_harness.c $(STANDIN)/graph_selftest.c
STANDIN_HDRS = $(wildcard $(STANDIN)/include/*.h $(STANDIN)/include/event2/*.h)
MOD_INC = -Iinclude -I$(MOD) -I$(STANDIN)/include
# grout's C flags (its meson.build) for the module's sources
MOD_CFLAGS = -std=gnu2x -D_GNU_SOURCE -DALLOW_EXPERIMENTAL_API -fms-extensions -Wmissing-prototypes -Wstrict-aliasing=2 \
	-fstrict-aliasing
HDRS = include/grout_hip.h $(CSRC)/fib6.h $(CSRC)/fwd4_kernel.h $(CSRC)/fwd4_dev.h $(CSRC)/fwd4_chain.h $(CSRC)/fib4.h

all: $(LIB_HIP) $(LIB_HOST) $(LIB_ORACLE) $(LIB_MOD) $(LIB_STANDIN) tools/libnode_mt.so

$(BUILD)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(BUILD)/gr_hip.o: $(CSRC)/gr_hip.cpp $(CSRC)/gr_node_priv.h $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(BUILD)/gr_node.o: $(CSRC)/gr_node.cpp $(CSRC)/gr_node_priv.h include/grout_hip.h
	@mkdir -p $(BUILD)
	$(CXX) -O3 -march=x86-64-v3 -fPIC -Wall -Wextra -std=c++17 -c -o $@ $<

$(BUILD)/fib4.o: $(CSRC)/fib4.c $(CSRC)/fib4.h
	@mkdir -p $(BUILD)
	$(CC) $(CFLAGS_HOST) -c -o $@ $<

$(BUILD)/fib6.o: $(CSRC)/fib6.c $(CSRC)/fib6.h
	@mkdir -p $(BUILD)
	$(CC) $(CFLAGS_HOST) -c -o $@ $<

$(LIB_HIP): $(BUILD)/fwd4_ring.o $(BUILD)/gr_hip.o $(BUILD)/gr_node.o $(BUILD)/fib4.o $(BUILD)/fib6.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^

$(LIB_HOST): $(CSRC)/fib4.c $(CSRC)/fib6.c $(CSRC)/synth.c $(CSRC)/fib4.h $(CSRC)/fib6.h $(CSRC)/synth.h include/grout_hip.h
	$(CC) $(CFLAGS_HOST) -shared -o $@ $(CSRC)/fib4.c $(CSRC)/fib6.c $(CSRC)/synth.c

$(LIB_ORACLE): oracle/oracle.c oracle/oracle.h include/grout_hip.h
	$(CC) $(CFLAGS_HOST) -pthread -shared -o $@ oracle/oracle.c

# links the HIP library (found next to it at run time)
$(LIB_MOD): $(MOD_SRC) $(MOD_HDRS) $(STANDIN_HDRS) $(LIB_HIP)
	$(CC) $(MOD_CFLAGS) $(CFLAGS_HOST) -pthread $(MOD_INC) -shared -o $@ $(MOD_SRC) -Lgrout_amd -lgrout_hip '-Wl,-rpath,$$ORIGIN'

$(LIB_STANDIN): $(STANDIN_SRC) $(STANDIN_HDRS) $(MOD_HDRS) $(LIB_MOD)
	$(CC) -std=gnu11 $(CFLAGS_HOST) -pthread $(MOD_INC) -shared -o $@ $(STANDIN_SRC) -Lgrout_amd -lgrout_gpu_fwd4 -lgrout_hip \
		'-Wl,-rpath,$$ORIGIN/../../grout_amd'

# measurement tool: the node walk from C threads (tools/node_pipeline.py --driver c)
tools/libnode_mt.so: tools/node_mt.c include/grout_hip.h $(LIB_HIP)
	$(CC) -O2 -pthread -fPIC -Wall -Iinclude -shared -o $@ $< -Lgrout_amd -lgrout_hip '-Wl,-rpath,$$ORIGIN/../grout_amd'

# ---- AddressSanitizer + UBSan build of the host code (CPU only) ----------
# Every host C/C++ source of the libraries and the oracle, built with the ROCm
# LLVM toolchain (hipcc's clang) so that one sanitizer runtime serves them
# all; the gfx950 kernel object is the normal one (no GPU sanitizer). The CPU
# test suite runs on these libraries with `make asan-test`.
LLVM = /opt/rocm/lib/llvm
ASAN_DIR = $(BUILD)/asan
ASAN_RT = $(firstword $(wildcard $(LLVM)/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so))
SAN = -fsanitize=address,undefined -fno-sanitize-recover=undefined -shared-libsan -fno-omit-frame-pointer -g -O1
SAN_C = $(LLVM)/bin/clang $(SAN) -fPIC -march=x86-64-v3 -Wall -Wno-unused-parameter
SAN_CXX = $(LLVM)/bin/clang++ $(SAN) -fPIC -march=x86-64-v3 -std=c++17 -Wall
SAN_HIP = $(HIPCC) -x hip --offload-arch=$(ARCH) -O1 -g -fPIC -std=c++17 -fno-omit-frame-pointer -Wno-unused-value \
	-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -shared-libsan

$(ASAN_DIR)/gr_hip.o: $(CSRC)/gr_hip.cpp $(HDRS)
	@mkdir -p $(ASAN_DIR)
	$(SAN_HIP) -c -o $@ $<

$(ASAN_DIR)/libgrout_hip.so: $(BUILD)/fwd4_ring.o $(ASAN_DIR)/gr_hip.o $(CSRC)/gr_node.cpp $(CSRC)/fib4.c $(CSRC)/fib6.c $(HDRS)
	$(SAN_C) -c -o $(ASAN_DIR)/fib4.o $(CSRC)/fib4.c
	$(SAN_C) -c -o $(ASAN_DIR)/fib6.o $(CSRC)/fib6.c
	$(SAN_CXX) -c -o $(ASAN_DIR)/gr_node.o $(CSRC)/gr_node.cpp
	$(SAN_CXX) -shared -o $@ $(BUILD)/fwd4_ring.o $(ASAN_DIR)/gr_hip.o $(ASAN_DIR)/gr_node.o \
		$(ASAN_DIR)/fib4.o $(ASAN_DIR)/fib6.o -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib

$(ASAN_DIR)/libgrout_host.so: $(CSRC)/fib4.c $(CSRC)/fib6.c $(CSRC)/synth.c $(CSRC)/fib4.h $(CSRC)/fib6.h $(CSRC)/synth.h
	@mkdir -p $(ASAN_DIR)
	$(SAN_C) -shared -o $@ $(CSRC)/fib4.c $(CSRC)/fib6.c $(CSRC)/synth.c

$(ASAN_DIR)/liboracle.so: oracle/oracle.c oracle/oracle.h include/grout_hip.h
	@mkdir -p $(ASAN_DIR)
	$(SAN_C) -pthread -shared -o $@ oracle/oracle.c

# globals not instrumented here: the identical edge-name literals of the node
# sources end up registered twice at one merged address (a false ODR report)
$(ASAN_DIR)/libgrout_gpu_fwd4.so: $(MOD_SRC) $(MOD_HDRS) $(STANDIN_HDRS) $(ASAN_DIR)/libgrout_hip.so
	$(SAN_C) -mllvm -asan-globals=0 -std=gnu11 $(MOD_INC) -shared -o $@ $(MOD_SRC) -L$(ASAN_DIR) -lgrout_hip '-Wl,-rpath,$$ORIGIN'

$(ASAN_DIR)/libgrout_standin.so: $(STANDIN_SRC) $(STANDIN_HDRS) $(MOD_HDRS) $(ASAN_DIR)/libgrout_gpu_fwd4.so
	$(SAN_C) -mllvm -asan-globals=0 -std=gnu11 $(MOD_INC) -shared -o $@ $(STANDIN_SRC) -L$(ASAN_DIR) -lgrout_gpu_fwd4 \
		-lgrout_hip '-Wl,-rpath,$$ORIGIN'

asan: $(ASAN_DIR)/libgrout_hip.so $(ASAN_DIR)/libgrout_host.so $(ASAN_DIR)/liboracle.so $(ASAN_DIR)/libgrout_standin.so

# the CPU suite on the sanitized libraries (GR_LIBDIR: abi.py / oracle load from there)
asan-test: asan
	GR_LIBDIR=$(ASAN_DIR) LD_PRELOAD=$(ASAN_RT) ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 \
		UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 python -m pytest tests -x -q -m "not gpu" -p no:cacheprovider

clean:
	rm -rf $(BUILD) $(LIB_HIP) $(LIB_HOST) $(LIB_ORACLE) $(LIB_MOD) $(LIB_STANDIN) grout_amd/libgrout_graph.so

.PHONY: all clean asan asan-test
