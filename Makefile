# Build the C-ABI shared library for gfx950 (MI355X).  Cross-compiles without a GPU.
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
SRC_DIR := notorch_amd/csrc
OUT     := notorch_amd/lib/libnotorch_amd.so
SRCS    := $(wildcard $(SRC_DIR)/*.hip)
OBJS    := $(patsubst $(SRC_DIR)/%.hip,build/%.o,$(SRCS))
HDRS    := $(wildcard $(SRC_DIR)/*.hpp) include/notorch_amd.h
FLAGS   := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-result \
           -fvisibility=hidden -DNT_BUILD

all: $(OUT)

build/%.o: $(SRC_DIR)/%.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(FLAGS) -c $< -o $@

$(OUT): $(OBJS)
	@mkdir -p $(dir $(OUT))
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -Wl,-rpath,/opt/rocm/lib

# resource usage report (VGPR / SGPR / LDS / occupancy) of every kernel
resource-usage: $(SRCS)
	@for f in $(SRCS); do $(HIPCC) $(FLAGS) -c $$f -o /dev/null -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "Function Name|VGPRs:|AGPRs|LDS Size|Occupancy|SGPRs:"; done

clean:
	rm -rf build $(OUT)

.PHONY: all clean resource-usage
