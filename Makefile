# Builds lesion_gnn_amd/liblgnn.so (gfx950 only). The oracle is Python (oracle/pyg_ref.py): nothing to compile.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function
SRC := $(wildcard lesion_gnn_amd/csrc/*.hip)
OBJ := $(patsubst lesion_gnn_amd/csrc/%.hip,build/%.o,$(SRC))
LIB := lesion_gnn_amd/liblgnn.so

all: $(LIB)

build/%.o: lesion_gnn_amd/csrc/%.hip $(wildcard lesion_gnn_amd/csrc/*.h) include/lgnn.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJ)
	$(HIPCC) $(HIPFLAGS) -shared $(OBJ) -o $@

resource-usage: $(SRC)
	@for f in $(SRC); do $(HIPCC) $(HIPFLAGS) -c $$f -o /dev/null -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "Function Name|VGPRs:|AGPRs|Spill|Occupancy|LDS Size" ; done

clean:
	rm -rf build $(LIB)

.PHONY: all clean resource-usage
