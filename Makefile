# Top-level build: the HIP engine (libmgicp.so, gfx950) and the CPU oracle (test infra).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH  ?= gfx950
PKG   := leica_point_cloud_processing_amd
LIB   := $(PKG)/libmgicp.so
SRCS  := $(PKG)/csrc/mgicp_kernels.hip $(PKG)/csrc/mgicp_engine.hip
HDRS  := $(wildcard $(PKG)/csrc/*.hpp) include/mi355x_gicp.h
# -ffp-contract=off: no FMA contraction, so fp32/fp64 expressions round like PCL's SSE2 Eigen
HIPFLAGS := -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -ffp-contract=off -Wall -Wno-unused-result

all: $(LIB) oracle adapter-example adapter-replay

OBJDIR := $(PKG)/csrc/build
OBJS  := $(OBJDIR)/mgicp_kernels.o $(OBJDIR)/mgicp_engine.o

# one object per source (make -j2 compiles both at once; an engine edit does not rebuild the kernels)
$(OBJDIR)/%.o: $(PKG)/csrc/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIB): $(OBJS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJS) -lrccl

# diagnostic builds: make variant NAME=diag DEFS=-DMGICP_CORR_PHASES=1 -> libmgicp_diag.so (MGICP_LIB_NAME selects it)
variant: $(SRCS) $(HDRS)
	$(HIPCC) $(HIPFLAGS) $(DEFS) -shared -o $(PKG)/libmgicp_$(NAME).so $(SRCS) -lrccl

# plain C++ host program over the C-ABI (g++, no HIP headers): what an integrator links
adapter/cabi_example: adapter/cabi_example.cpp include/mi355x_gicp.h $(LIB)
	g++ -O2 -std=c++14 -Wall -Iinclude -o $@ adapter/cabi_example.cpp -L$(PKG) -lmgicp -Wl,-rpath,'$$ORIGIN/../$(PKG)'

adapter-example: adapter/cabi_example

# the drop-in adapter itself (adapter/GICPAlignment.cpp + adapter/Filter_mi355x.cpp), compiled as the
# catkin package would compile it (-std=c++14, the reference's CMakeLists.txt:6) against the
# layout-exact PCL / Eigen / ROS stand-ins of tests/adapter_standins (PCL and ROS are absent here),
# linked with a replay of test/test_gicp_alignment.cpp:50-131 (test infrastructure)
STANDIN := tests/adapter_standins
REPLAY  := adapter/build/replay_test_gicp_alignment
$(REPLAY): adapter/GICPAlignment.cpp adapter/GICPAlignment.h adapter/Filter_mi355x.cpp include/mi355x_gicp.h \
           $(wildcard $(STANDIN)/*.h) $(STANDIN)/Utils_standin.cpp $(STANDIN)/replay_test_gicp_alignment.cpp $(LIB)
	mkdir -p adapter/build
	g++ -O2 -std=c++14 -Wall -Wextra -Werror -I$(STANDIN) -Iadapter -Iinclude -o $@ \
	    adapter/GICPAlignment.cpp adapter/Filter_mi355x.cpp $(STANDIN)/Utils_standin.cpp \
	    $(STANDIN)/replay_test_gicp_alignment.cpp -L$(PKG) -lmgicp -Wl,-rpath,'$$ORIGIN/../../$(PKG)'

adapter-replay: $(REPLAY)

oracle:
	$(MAKE) -C oracle

clean:
	rm -f $(LIB) $(PKG)/libmgicp_*.so $(OBJS)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean adapter-example adapter-replay variant
