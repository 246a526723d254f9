# Build of the MI355X (gfx950) engine and the CPU checkers.  No cmake/ninja needed.
#
#   make            -> seqalib_amd/lib/libseqalib_hip.so  (HIP kernels + C ABI)
#   make oracle     -> oracle/liboracle.so                (C restatement, test infrastructure)
#   make ref        -> oracle/_ref/libsaref.so            (reference built in place; needs /root/reference)
#   make all-checkers / clean

HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result
CSRC      = seqalib_amd/csrc
OBJDIR    = build/obj
LIB       = seqalib_amd/lib/libseqalib_hip.so

HIP_SRCS  = $(CSRC)/sa_fill_sw.hip $(CSRC)/sa_fill_so2.hip $(CSRC)/sa_fill_nw.hip $(CSRC)/sa_fill_lg.hip $(CSRC)/sa_fill_gg.hip \
            $(CSRC)/sa_traceback.hip $(CSRC)/sa_traceback_so.hip $(CSRC)/sa_traceback_wave.hip $(CSRC)/sa_traceback_seg.hip $(CSRC)/sa_alphabet.hip $(CSRC)/sa_endcell.hip $(CSRC)/sa_hirschberg.hip $(CSRC)/sa_dc.hip \
            $(CSRC)/sa_myersmiller.hip $(CSRC)/sa_tiny.hip $(CSRC)/sa_api.hip
CPP_SRCS  = $(CSRC)/sa_synth.cpp $(CSRC)/sa_multi.cpp $(CSRC)/sa_codec.cpp
HDRS      = $(CSRC)/sa_internal.h $(CSRC)/sa_layout.h $(CSRC)/sa_fill_impl.h $(CSRC)/sa_dc.h include/seqalib_hip.h
OBJS      = $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.o,$(HIP_SRCS)) $(patsubst $(CSRC)/%.cpp,$(OBJDIR)/%.o,$(CPP_SRCS))

lib: $(LIB)

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	@mkdir -p $(dir $@)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(OBJS) -lpthread

# debug build with traceback / SPLIT counters (tools/tb_stats.py, tools/split_stats.py):
# build/libstats.so, copied to tools/bin/ (build/ does not travel to the GPU box)
STATS_LIB = build/libstats.so
stats: $(STATS_LIB)
$(STATS_LIB): $(HIP_SRCS) $(CPP_SRCS) $(HDRS)
	@mkdir -p build/stats
	printf '%s\n' $(HIP_SRCS) $(CPP_SRCS) | xargs -P 8 -I{} sh -c '$(HIPCC) $(HIPFLAGS) -DSA_TB_STATS -c {} -o build/stats/$$(basename {}).o'
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ build/stats/*.o -lpthread
	@mkdir -p tools/bin && cp $@ tools/bin/libstats.so

oracle:
	$(MAKE) -C oracle

ref:
	$(MAKE) -C oracle ref

all-checkers: oracle ref

clean:
	rm -rf build $(LIB)
	$(MAKE) -C oracle clean

# A/B variant of the engine: make variant V=name DEFS="-DSOMETHING" -> seqalib_amd/lib/ab/lib<name>.so
variant:
	@mkdir -p build/ab_$(V) seqalib_amd/lib/ab
	printf '%s\n' $(HIP_SRCS) $(CPP_SRCS) | xargs -P 8 -I{} sh -c '$(HIPCC) $(HIPFLAGS) $(DEFS) -c {} -o build/ab_$(V)/$$(basename {}).o'
	$(HIPCC) -shared --offload-arch=$(ARCH) -o seqalib_amd/lib/ab/lib$(V).so build/ab_$(V)/*.o -lpthread

.PHONY: lib stats variant oracle ref all-checkers clean
