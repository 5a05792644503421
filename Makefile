# Build the C-ABI shared library for gfx950 (MI355X).  Cross-compiles without a GPU.
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
SRC_DIR := notorch_amd/csrc
SRCS    := $(wildcard $(SRC_DIR)/*.hip)
HDRS    := $(wildcard $(SRC_DIR)/*.hpp) $(wildcard $(SRC_DIR)/diag/*.hpp) include/notorch_amd.h
FLAGS   := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-result \
           -fvisibility=hidden -DNT_BUILD
# DIAG=1: the diagnostic library (A/B kernel variants, ablation and stamp builds selected by NT_*
# environment variables) next to the shipping one; notorch_amd._lib loads it when NT_LIB=diag.
# VARIANT=<name> EXTRA=-D...: an A/B build of the shipping sources into lib/libnotorch_amd_<name>.so
# (loaded with NT_LIB=variant:<name>; experiments only, git- and gpurun-ignored build dirs)
FLAGS   += $(EXTRA)
ifeq ($(DIAG),1)
OUT     := notorch_amd/lib/libnotorch_amd_diag.so
BDIR    := build_diag
FLAGS   += -DNT_DIAG
# csrc/diag/: kernels of the diagnostic library only (A/B variants superseded in the shipping one)
SRCS    += $(wildcard $(SRC_DIR)/diag/*.hip)
else ifneq ($(VARIANT),)
OUT     := notorch_amd/lib/libnotorch_amd_$(VARIANT).so
BDIR    := build_$(VARIANT)
else
OUT     := notorch_amd/lib/libnotorch_amd.so
BDIR    := build
endif
OBJS    := $(patsubst $(SRC_DIR)/%.hip,$(BDIR)/%.o,$(SRCS))
DIAG_OBJS := $(filter $(BDIR)/diag/%,$(OBJS))

# host-only CPython helper of the native collate (csrc/host/collate_py.cpp): g++ against torch's headers
PY      ?= python3
PYEXT   := notorch_amd/lib/_collate_py$(shell $(PY) -c "import sysconfig; print(sysconfig.get_config_var('EXT_SUFFIX'))")
TORCH_FLAGS = $(shell $(PY) -c "import sysconfig, os, torch, torch.utils.cpp_extension as c; \
  print(' '.join('-I' + p for p in c.include_paths()), '-I' + sysconfig.get_paths()['include'], \
  '-D_GLIBCXX_USE_CXX11_ABI=%d' % int(torch._C._GLIBCXX_USE_CXX11_ABI), \
  '-L' + os.path.join(os.path.dirname(torch.__file__), 'lib'))")

ifeq ($(DIAG)$(VARIANT),)
all: $(OUT) $(PYEXT)
else
all: $(OUT)
endif

$(PYEXT): $(SRC_DIR)/host/collate_py.cpp
	@mkdir -p $(dir $@)
	g++ -O3 -std=c++17 -shared -fPIC -Wall $(TORCH_FLAGS) $< -o $@ -ltorch_python -ltorch_cpu -lc10

$(BDIR)/%.o: $(SRC_DIR)/%.hip $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(FLAGS) -c $< -o $@

$(OUT): $(OBJS)
	@mkdir -p $(dir $(OUT))
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -Wl,-rpath,/opt/rocm/lib

# resource usage report (VGPR / SGPR / LDS / occupancy) of every kernel
resource-usage: $(SRCS)
	@for f in $(SRCS); do $(HIPCC) $(FLAGS) -c $$f -o /dev/null -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "Function Name|VGPRs:|AGPRs|LDS Size|Occupancy|SGPRs:"; done

clean:
	rm -rf build build_diag notorch_amd/lib/libnotorch_amd.so notorch_amd/lib/libnotorch_amd_diag.so $(PYEXT)

.PHONY: all clean resource-usage
