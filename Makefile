# Build of the MI355X (gfx950) candidate scorer — in-tree, no cmake.
#   make            -> sspp_amd/lib/libsspp_hip.so + sspp/_sspp*.so (pybind11 drop-in) + oracle
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
PY       ?= python3
JOBS     ?= 8
CXXSTD    = -std=c++17
# -ffp-contract=off: every fma in the kernels is explicit (bitwise parity with oracle/)
HIPFLAGS  = $(CXXSTD) -O3 -fPIC --offload-arch=$(ARCH) -ffp-contract=off -fno-fast-math \
            -Wall -Wno-unused-function -Wno-unused-result $(EXTRA)
HOSTFLAGS = $(CXXSTD) -O2 -fPIC -ffp-contract=off -Wall -mfma

SRC      = sspp_amd/csrc
LIBDIR   = sspp_amd/lib
OBJDIR   = build/obj
LIB      = $(LIBDIR)/libsspp_hip.so
PYEXT    = $(shell $(PY) -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
PYMOD    = sspp/_sspp$(PYEXT)
PYMOD2   = sspp/_tsp$(PYEXT)
PYINC    = $(shell $(PY) -c "import sysconfig;print(sysconfig.get_paths()['include'])")
PBINC    = $(shell $(PY) -c "import pybind11;print(pybind11.get_include())")

HDRS = include/sspp_hip.h $(SRC)/sspp_logtab.h $(SRC)/model.h $(SRC)/sspp_device.h $(SRC)/sspp_filter.h $(SRC)/xml_lite.h $(SRC)/sspp_kern.h
# kernel instantiations, one translation unit per (dof, degree) (+ d0: TaskSpacePlanner), compiled
# in parallel (one unit per degree also keeps the register allocation of each kernel its own)
INST = $(OBJDIR)/sspp_inst_d0.o $(foreach d,1 2 3 4 6 7 9,$(foreach p,2 3,$(OBJDIR)/sspp_inst_d$(d)_p$(p).o))

all: $(LIB) $(PYMOD) $(PYMOD2) oracle

$(OBJDIR)/%.o: $(SRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HOSTFLAGS) -c $< -o $@

$(OBJDIR)/%.o: $(SRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/sspp_inst_d0.o: $(SRC)/sspp_inst.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -DSSPK_D=0 -c $< -o $@

$(OBJDIR)/sspp_inst_d%.o: $(SRC)/sspp_inst.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -DSSPK_D=$(firstword $(subst _p, ,$*)) -DSSPK_P=$(lastword $(subst _p, ,$*)) -c $< -o $@

# the source revision, compiled in as sspp_build_id() (sspp_amd/_stamp.py; checked at load time
# by sspp_amd/_lib.py): rebuilt whenever any source changes
SRCS = $(wildcard $(SRC)/*.h $(SRC)/*.hip $(SRC)/*.cpp) include/sspp_hip.h
$(OBJDIR)/stamp.o: $(SRCS) sspp_amd/_stamp.py
	@mkdir -p $(OBJDIR)
	@printf 'extern "C" const char* sspp_build_id() { return "%s"; }\n' `$(PY) sspp_amd/_stamp.py` > $(OBJDIR)/stamp.cpp
	g++ $(HOSTFLAGS) -c $(OBJDIR)/stamp.cpp -o $@

$(LIB): $(OBJDIR)/sspp_kernels.o $(INST) $(OBJDIR)/ces.o $(OBJDIR)/planner.o $(OBJDIR)/sspp_capi.o $(OBJDIR)/mjcf.o $(OBJDIR)/spline_host.o $(OBJDIR)/sspp_hostapi.o $(OBJDIR)/stamp.o
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^

$(PYMOD): $(SRC)/sspp_pybind.cpp $(LIB) include/sspp_hip.h
	g++ $(CXXSTD) -O2 -fPIC -shared -I$(PYINC) -I$(PBINC) -Iinclude $< -o $@ \
	    -L$(LIBDIR) -lsspp_hip -Wl,-rpath,'$$ORIGIN/../sspp_amd/lib'

$(PYMOD2): $(SRC)/tsp_pybind.cpp $(LIB) include/sspp_hip.h
	g++ $(CXXSTD) -O2 -fPIC -shared -I$(PYINC) -I$(PBINC) -Iinclude $< -o $@ \
	    -L$(LIBDIR) -lsspp_hip -Wl,-rpath,'$$ORIGIN/../sspp_amd/lib'

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf build $(LIB) $(PYMOD) $(PYMOD2)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean
