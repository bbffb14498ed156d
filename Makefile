# Builds the MI355X (gfx950) engine library and the CPU oracle.  `python -c "import
# __graft_entry__ as g; g.build()"` runs the same steps.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function
CSRC := sdfs_amd/csrc
LIB := sdfs_amd/libsdfs_cdc.so
OBJS := build/cdc_kernels.o build/cdc_engine.o build/dedup_index.o build/lz4_kernels.o build/map_emit.o build/aes_kernels.o
SWEEP_LIB := sdfs_amd/libsdfs_cdc_sweep.so

all: $(LIB) oracle

# kernel-variant sweep build (scripts/sweep_scan.py); not used by the product path
sweep: $(SWEEP_LIB)
build/sweep_kernels.o: $(CSRC)/cdc_kernels.hip $(CSRC)/cdc_internal.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -DSDFS_SCAN_SWEEP -c $< -o $@
$(SWEEP_LIB): build/sweep_kernels.o build/cdc_engine.o build/dedup_index.o build/lz4_kernels.o build/map_emit.o build/aes_kernels.o
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $^

build/%.o: $(CSRC)/%.hip $(CSRC)/cdc_internal.h include/sdfs_cdc.h include/sdfs_index.h include/sdfs_lz4.h include/sdfs_meta.h include/sdfs_aes.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJS)

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf build $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean sweep
