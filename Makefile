# Builds the MI355X (gfx950) engine library, the measurement (tuning) library and the CPU
# oracle.  `python -c "import __graft_entry__ as g; g.build()"` runs the same steps.
#   sdfs_amd/libsdfs_cdc.so         the product: production kernels only, reads no environment
#   sdfs_amd/libsdfs_cdc_tuning.so  the same C-ABI plus the measured kernel variants and the
#                                   SDFS_* A/B switches (-DSDFS_TUNING; scripts/, variant tests)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function
CSRC := sdfs_amd/csrc
LIB := sdfs_amd/libsdfs_cdc.so
TUNING_LIB := sdfs_amd/libsdfs_cdc_tuning.so
SRCS := cdc_kernels cdc_engine dedup_index lz4_kernels map_emit aes_kernels
OBJS := $(SRCS:%=build/%.o)
TUNING_OBJS := $(SRCS:%=build/tuning/%.o) build/tuning/cdc_sweep.o build/tuning/cdc_sweep_r3.o
HDRS := $(CSRC)/cdc_internal.h $(CSRC)/cdc_device.h $(CSRC)/host_queue.h $(CSRC)/engine_share.h $(CSRC)/stream_order.h $(wildcard include/*.h)

all: $(LIB) tuning tools oracle buildinfo

# the commit the built libraries come from (bench.py reports it; the GPU box has no .git)
buildinfo:
	@git rev-parse --short=12 HEAD > sdfs_amd/BUILD_COMMIT 2>/dev/null && (git diff --quiet HEAD -- sdfs_amd include 2>/dev/null || sed -i 's/$$/+dirty/' sdfs_amd/BUILD_COMMIT) || true

tuning: $(TUNING_LIB)

build/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/tuning/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p build/tuning
	$(HIPCC) $(HIPFLAGS) -DSDFS_TUNING -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) $(HIPFLAGS) -shared -Wl,-z,defs -o $@ $(OBJS) -ldl

$(TUNING_LIB): $(TUNING_OBJS)
	$(HIPCC) $(HIPFLAGS) -shared -Wl,-z,defs -o $@ $(TUNING_OBJS) -ldl

# host-side harnesses: the multi-threaded getChunks driver (bench.py, GPU tests) and the JNI glue
tools: tools/libsdfs_threads.so tools/libsdfs_threads_tuning.so tools/libsdfs_probe.so jni/libsdfs_cdc_jni.so tests/jni/libjni_stub.so

tools/libsdfs_threads.so: tools/threads_bench.c include/sdfs_cdc.h $(LIB)
	gcc -O2 -std=c11 -fPIC -shared -Wl,-z,defs -Wall -Wextra -D_GNU_SOURCE -o $@ $< -Lsdfs_amd -lsdfs_cdc -Wl,-rpath,'$$ORIGIN/../sdfs_amd' -lpthread

# the same harness against the tuning library (scripts/ with SDFS_CDC_LIB=...tuning.so: an engine
# handle is only valid in the library that made it)
tools/libsdfs_threads_tuning.so: tools/threads_bench.c include/sdfs_cdc.h $(TUNING_LIB)
	gcc -O2 -std=c11 -fPIC -shared -Wl,-z,defs -Wall -Wextra -D_GNU_SOURCE -o $@ $< -Lsdfs_amd -lsdfs_cdc_tuning -Wl,-rpath,'$$ORIGIN/../sdfs_amd' -lpthread

# measurement-only kernels bench.py runs beside the product library (the fingerprint's VALU ceiling)
tools/libsdfs_probe.so: tools/probe_kernels.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -shared -Wl,-z,defs -o $@ $<

jni/libsdfs_cdc_jni.so: jni/sdfs_cdc_jni.c jni/jni_min.h include/sdfs_cdc.h $(LIB)
	gcc -O2 -std=c11 -fPIC -shared -Wl,-z,defs -Wall -Wextra -o $@ $< -Lsdfs_amd -lsdfs_cdc -Wl,-rpath,'$$ORIGIN/../sdfs_amd'

# test infrastructure: a stand-in JNIEnv for driving the JNI glue without a JVM (tests/test_jni.py)
tests/jni/libjni_stub.so: tests/jni/jni_stub.c jni/jni_min.h
	gcc -O2 -std=gnu11 -fPIC -shared -Wall -Wextra -o $@ $<

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf build $(LIB) $(TUNING_LIB) tools/*.so jni/*.so tests/jni/*.so
	$(MAKE) -C oracle clean

.PHONY: all oracle clean tuning tools buildinfo
