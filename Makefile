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
LIB_GRAPH = grout_amd/libgrout_graph.so
GRAPH = grout_amd/graph
GRAPH_SRC = $(GRAPH)/rte_graph_min.c $(GRAPH)/gr_datapath_min.c $(GRAPH)/gpu_fwd4_node.c $(GRAPH)/walk_harness.c \
	$(GRAPH)/graph_selftest.c
GRAPH_HDRS = $(GRAPH)/rte_graph_min.h $(GRAPH)/gr_datapath_min.h $(GRAPH)/gpu_fwd4_node.h include/grout_hip.h
HDRS = include/grout_hip.h $(CSRC)/fib6.h $(CSRC)/fwd4_kernel.h $(CSRC)/fwd4_dev.h $(CSRC)/fwd4_chain.h $(CSRC)/fib4.h

all: $(LIB_HIP) $(LIB_HOST) $(LIB_ORACLE) $(LIB_GRAPH)

$(BUILD)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(BUILD)/gr_hip.o: $(CSRC)/gr_hip.cpp $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(BUILD)/gr_node.o: $(CSRC)/gr_node.cpp include/grout_hip.h
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

# The fast path's grout node (C) on the rte_graph / grout stand-ins, with the
# test harness graph; links the HIP library (found next to it at run time).
$(LIB_GRAPH): $(GRAPH_SRC) $(GRAPH_HDRS) $(LIB_HIP)
	$(CC) -std=gnu11 $(CFLAGS_HOST) -Iinclude -shared -o $@ $(GRAPH_SRC) -Lgrout_amd -lgrout_hip '-Wl,-rpath,$$ORIGIN'

clean:
	rm -rf $(BUILD) $(LIB_HIP) $(LIB_HOST) $(LIB_ORACLE) $(LIB_GRAPH)

.PHONY: all clean
