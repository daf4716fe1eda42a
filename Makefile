# Build of the MI355X-native RS coding path (gfx950 only).
#   make            -> nexoedge_amd/lib/libnxec.so (+ C++ coding surface) and oracle/liboracle.so
#   make ref        -> oracle/_ref (reference ISA-L base C, needs /root/reference; build container only)
#   make golden     -> regenerate tests/golden/golden.json from oracle/_ref
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
CXXSTD   := -std=c++17
# PROBES=1 adds the design-probe kernels (DESIGN.md section 4 A/Bs; `make clean` first)
PROBES   ?= 0
HIPFLAGS := --offload-arch=$(ARCH) -O3 -fPIC $(CXXSTD) -Wall -Iinclude -Inexoedge_amd/csrc \
            -mllvm -amdgpu-atomic-optimizer-strategy=None -DNXEC_DESIGN_PROBES=$(PROBES) $(EXTRA_FLAGS)
LIBDIR   := nexoedge_amd/lib
CSRC     := nexoedge_amd/csrc
OBJDIR   := build/obj

LIB_SRCS := $(CSRC)/gf_host.cpp $(CSRC)/nxec_context.cpp $(CSRC)/nxec_stripes.cpp $(CSRC)/nxec_objects.cpp \
            $(CSRC)/nxec_host_paths.cpp $(CSRC)/nxec_host_encode.cpp $(CSRC)/nxec_agent.cpp $(CSRC)/nxec_probes.cpp \
            $(CSRC)/nxec_kernels.hip $(CSRC)/nxec_md5.hip $(CSRC)/nxec_encode_md5.hip $(CSRC)/nxec_encode_md5_ring.hip \
            $(CSRC)/nxec_files_md5.hip \
            $(CSRC)/nxec_group.cpp $(CSRC)/nxec_host_arena.cpp $(CSRC)/nxec_digest.cpp $(CSRC)/nxec_digest_place.cpp $(CSRC)/nxec_numa.cpp $(CSRC)/nxec_config.cpp \
            $(CSRC)/coding/rs.cc $(CSRC)/coding/coding_options.cc $(CSRC)/coding/stripe_batch.cc
LIB_OBJS := $(patsubst $(CSRC)/%,$(OBJDIR)/%.o,$(LIB_SRCS))
HDRS     := include/nxec.h $(CSRC)/nxec_internal.h $(CSRC)/nxec_runtime.h $(CSRC)/nxec_tuning.h $(CSRC)/nxec_device.h $(CSRC)/nxec_em_common.h $(wildcard $(CSRC)/coding/*.hh)

all: $(LIBDIR)/libnxec.so oracle/liboracle.so build/rs_surface_test build/isal_compat_test build/chunk_manager_flow_test \
     build/stripe_batch_test build/chunk_replay_test build/dropin_pool_test

# rs.cc's ISA-L call sequence compiled against include/nxec_isal_compat.h (plain C)
build/isal_compat_test: tests/cpp/isal_compat_test.c include/nxec_isal_compat.h $(LIBDIR)/libnxec.so
	@mkdir -p build
	gcc -std=c11 -O2 -Wall -Iinclude $< -L$(LIBDIR) -lnxec -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)' -lcrypto -o $@

# C++ surface test (reference coding_test.cc flows through RSCode on the GPU)
build/rs_surface_test: tests/cpp/rs_surface_test.cc $(LIBDIR)/libnxec.so $(HDRS)
	@mkdir -p build
	g++ -std=c++17 -O2 -Wall -Iinclude -I$(CSRC) $< -L$(LIBDIR) -lnxec -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)' -lcrypto -o $@

# batched ChunkManager entry vs the per-stripe RSCode path
build/stripe_batch_test: tests/cpp/stripe_batch_test.cc $(LIBDIR)/libnxec.so $(HDRS)
	@mkdir -p build
	g++ -std=c++17 -O2 -Wall -Iinclude -I$(CSRC) $< -L$(LIBDIR) -lnxec -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)' -lcrypto -o $@

# the default pool under 16 proxy workers sharing one RSCode (oracle = checker only)
build/dropin_pool_test: tests/cpp/dropin_pool_test.cc $(LIBDIR)/libnxec.so oracle/liboracle.so $(HDRS)
	@mkdir -p build
	g++ -std=c++17 -O2 -Wall -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -I$(CSRC) $< -L$(LIBDIR) -lnxec \
	    -Loracle -loracle -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)' -Wl,-rpath,'$$ORIGIN/../oracle' \
	    -Wl,-rpath,/opt/rocm/lib -lcrypto -lpthread -o $@

# the reference's Chunk ownership sequences (shallow copies + freeData = false)
build/chunk_replay_test: tests/cpp/chunk_replay_test.cc $(LIBDIR)/libnxec.so $(HDRS)
	@mkdir -p build
	g++ -std=c++17 -O2 -Wall -Iinclude -I$(CSRC) $< -L$(LIBDIR) -lnxec -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)' -lcrypto -o $@

# unmodified-ChunkManager repair flow: CodingOptions() fed by the Config bridge
# (nexoedge_amd/integration/nxec_config_bridge.cc) over a test double of Config
STUB := tests/cpp/nexoedge_stub/common
build/chunk_manager_flow_test: tests/cpp/chunk_manager_flow_test.cc nexoedge_amd/integration/nxec_config_bridge.cc \
                               $(STUB)/config.hh $(LIBDIR)/libnxec.so $(HDRS)
	@mkdir -p build
	g++ -std=c++17 -O2 -Wall -Iinclude -I$(CSRC) -I$(CSRC)/coding -I$(STUB) -I$(STUB)/coding \
	    tests/cpp/chunk_manager_flow_test.cc nexoedge_amd/integration/nxec_config_bridge.cc \
	    -L$(LIBDIR) -lnxec -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)' -lcrypto -o $@

$(OBJDIR)/%.o: $(CSRC)/% $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/libnxec.so: $(LIB_OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(LIB_OBJS) -lcrypto -o $@

oracle/liboracle.so: oracle/nxec_oracle.c oracle/nxec_cpu_simd.c oracle/nxec_oracle.h
	gcc -O2 -std=c11 -Wall -fPIC -shared oracle/nxec_oracle.c oracle/nxec_cpu_simd.c -o $@ -lpthread

# drop-in per-stripe rate through the C++ surface (tools/dropin_rate.cc)
tools: build/dropin_rate
build/dropin_rate: tools/dropin_rate.cc $(LIBDIR)/libnxec.so $(HDRS)
	@mkdir -p build
	g++ -std=c++17 -O2 -Wall -Iinclude -I$(CSRC) $< -L$(LIBDIR) -lnxec -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)' -lcrypto -lpthread -o $@

# design probes (not product): LDS-table variants and memory-side tuning vs the product kernel
tune: tools/microbench/tune_mul tools/microbench/lut_variants tools/microbench/shape_ceiling tools/microbench/mem_pattern tools/microbench/chunk_stride
tools/microbench/shape_ceiling: tools/microbench/shape_ceiling.hip $(LIBDIR)/libnxec.so
	$(HIPCC) --offload-arch=$(ARCH) -O3 -Iinclude $< -L$(LIBDIR) -lnxec -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -o $@
tools/microbench/tune_mul: tools/microbench/tune_mul.hip $(LIBDIR)/libnxec.so
	$(HIPCC) --offload-arch=$(ARCH) -O3 -Iinclude $< -L$(LIBDIR) -lnxec -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -o $@
tools/microbench/mem_pattern: tools/microbench/mem_pattern.hip $(LIBDIR)/libnxec.so
	$(HIPCC) --offload-arch=$(ARCH) -O3 -Iinclude $< -L$(LIBDIR) -lnxec -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -o $@
tools/microbench/chunk_stride: tools/microbench/chunk_stride.hip $(LIBDIR)/libnxec.so
	$(HIPCC) --offload-arch=$(ARCH) -O3 -Iinclude $< -L$(LIBDIR) -lnxec -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -o $@
tools/microbench/lut_variants: tools/microbench/lut_variants.hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 $< -o $@

# ---- sanitizer builds of the host code (CPU only; SURVEY §5, reference
# CMakeLists.txt:37-39).  Every source is compiled with the sanitizer on the
# host side only (-Xarch_host; the device code is the normal gfx950 build and
# these builds never launch a kernel: they run where no GPU is visible), then
# tests/cpp/host_sanity_test.cc drives planning, argument
# validation, the CodingOptions defaults source, Chunk/arena ownership and the
# host worker pool from 8 threads.  `make sanitize` builds and runs all three.
SAN_ASAN  := -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer
SAN_UBSAN := -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined
SAN_TSAN  := -Xarch_host -fsanitize=thread
SAN_CFLAGS = --offload-arch=$(ARCH) -O1 -g -fPIC $(CXXSTD) -Iinclude -I$(CSRC) \
             -mllvm -amdgpu-atomic-optimizer-strategy=None
SAN_SRCS := $(LIB_SRCS)
define SAN_RULES
build/san/$(1)/obj/%.o: $(CSRC)/% $(HDRS)
	@mkdir -p $$(dir $$@)
	$(HIPCC) $(SAN_CFLAGS) $(2) -c $$< -o $$@
build/san/$(1)/libnxec.so: $(patsubst $(CSRC)/%,build/san/$(1)/obj/%.o,$(SAN_SRCS))
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(2) $$^ -lcrypto -o $$@
build/san/$(1)/host_sanity_test: tests/cpp/host_sanity_test.cc build/san/$(1)/libnxec.so $(HDRS)
	$(HIPCC) -O1 -g $(CXXSTD) $(2) -Iinclude -I$(CSRC) $$< -Lbuild/san/$(1) -lnxec \
	    -Wl,-rpath,'$$$$ORIGIN' -lcrypto -lpthread -o $$@
build/san/$(1)/chunk_replay_test: tests/cpp/chunk_replay_test.cc build/san/$(1)/libnxec.so $(HDRS)
	$(HIPCC) -O1 -g $(CXXSTD) $(2) -Iinclude -I$(CSRC) $$< -Lbuild/san/$(1) -lnxec \
	    -Wl,-rpath,'$$$$ORIGIN' -lcrypto -lpthread -o $$@
$(1): build/san/$(1)/host_sanity_test build/san/$(1)/chunk_replay_test
endef
$(eval $(call SAN_RULES,asan,$(SAN_ASAN)))
$(eval $(call SAN_RULES,ubsan,$(SAN_UBSAN)))
$(eval $(call SAN_RULES,tsan,$(SAN_TSAN)))
sanitize: asan ubsan tsan
	ASAN_OPTIONS=detect_leaks=1 LSAN_OPTIONS=suppressions=tests/cpp/lsan.supp build/san/asan/host_sanity_test
	ASAN_OPTIONS=detect_leaks=1 LSAN_OPTIONS=suppressions=tests/cpp/lsan.supp build/san/asan/chunk_replay_test
	UBSAN_OPTIONS=print_stacktrace=1 build/san/ubsan/host_sanity_test
	TSAN_OPTIONS=ignore_noninstrumented_modules=1 build/san/tsan/host_sanity_test

ref:
	bash oracle/build_ref.sh

golden: ref
	oracle/_ref/gen_golden > tests/golden/golden.json

clean:
	rm -rf build $(LIBDIR)/libnxec.so oracle/liboracle.so

.PHONY: all ref golden clean tune tools asan ubsan tsan sanitize
