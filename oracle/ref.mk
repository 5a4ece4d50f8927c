# oracle/ref.mk — builds the REFERENCE (VTM 7.3, /root/reference) from its own sources, in place,
# with plain g++ (no cmake, no generated code, no external libraries). TEST INFRASTRUCTURE ONLY:
# everything lands in oracle/_ref/ (git-ignored). Nothing here is part of the product path.
#
#   make -f oracle/ref.mk -j8            # DecoderApp, EncoderApp, vtm_capture
#
# Flags mirror the reference's Release configuration (CMakeLists.txt:40-41 c++11, :104-106 -msse4.1,
# source/Lib/CommonLib/CMakeLists.txt:88-102 per-ISA defines/flags, :85 include dirs).

REF      ?= /root/reference
OUT      ?= $(CURDIR)/oracle/_ref
SRC       = $(REF)/source
CXX      ?= g++
CXXFLAGS  = -O3 -std=c++11 -fPIC -msse4.1 -DNDEBUG -w -pthread \
            -DENABLE_SPLIT_PARALLELISM=0 -DENABLE_WPP_PARALLELISM=0 \
            -I$(SRC)/Lib -I$(SRC)/Lib/CommonLib -I$(SRC)/Lib/CommonLib/x86 -I$(SRC)/Lib/libmd5 \
            -I$(SRC)/Lib/DecoderLib -I$(SRC)/Lib/EncoderLib -I$(SRC)/Lib/Utilities $(EXTRA)

COMMON_SRC = $(wildcard $(SRC)/Lib/CommonLib/*.cpp) $(wildcard $(SRC)/Lib/CommonLib/x86/*.cpp) \
             $(wildcard $(SRC)/Lib/libmd5/*.cpp)
SSE41_SRC  = $(wildcard $(SRC)/Lib/CommonLib/x86/sse41/*.cpp)
SSE42_SRC  = $(wildcard $(SRC)/Lib/CommonLib/x86/sse42/*.cpp)
AVX_SRC    = $(wildcard $(SRC)/Lib/CommonLib/x86/avx/*.cpp)
AVX2_SRC   = $(wildcard $(SRC)/Lib/CommonLib/x86/avx2/*.cpp)
DEC_SRC    = $(wildcard $(SRC)/Lib/DecoderLib/*.cpp)
ENC_SRC    = $(wildcard $(SRC)/Lib/EncoderLib/*.cpp)
UTIL_SRC   = $(wildcard $(SRC)/Lib/Utilities/*.cpp)
DECAPP_SRC = $(wildcard $(SRC)/App/DecoderApp/*.cpp)
ENCAPP_SRC = $(wildcard $(SRC)/App/EncoderApp/*.cpp)

obj = $(patsubst $(SRC)/%.cpp,$(OUT)/obj/%.o,$(1))

COMMON_OBJ = $(call obj,$(COMMON_SRC) $(SSE41_SRC) $(SSE42_SRC) $(AVX_SRC) $(AVX2_SRC))
DEC_OBJ    = $(call obj,$(DEC_SRC))
ENC_OBJ    = $(call obj,$(ENC_SRC))
UTIL_OBJ   = $(call obj,$(UTIL_SRC))
DECAPP_OBJ = $(call obj,$(DECAPP_SRC))
ENCAPP_OBJ = $(call obj,$(ENCAPP_SRC))

# link-time interposition used by the capture tool (GNU ld --wrap): every reference function whose
# result we record as a golden vector. Calls from DecCu.o / DecLib.o into these land in
# oracle/capture/vtm_capture.cpp, which calls the real function and records in/out.
WRAPS = $(shell cat $(CURDIR)/oracle/capture/wraps.txt 2>/dev/null)
WRAPFLAGS = $(foreach s,$(WRAPS),-Wl,--wrap=$(s))

all: apps capture rdo_kat mc_kat $(if $(wildcard $(CURDIR)/vvc_amd/libvvcr.so),dropin encdropin)

# syntax-trace decoder (the reference's own ENABLE_TRACING / DTRACE build, TypeDef.h) for debugging the
# host parser element by element: make -f oracle/ref.mk trace  ->  oracle/_ref/trace/DecoderApp
trace:
	$(MAKE) -f $(CURDIR)/oracle/ref.mk OUT=$(OUT)/trace EXTRA=-DENABLE_TRACING=1 $(OUT)/trace/DecoderApp
apps: $(OUT)/DecoderApp $(OUT)/EncoderApp
capture: $(OUT)/vtm_capture

$(OUT)/libCommonLib.a: $(COMMON_OBJ)
	@mkdir -p $(@D); rm -f $@; ar rcs $@ $^
$(OUT)/libDecoderLib.a: $(DEC_OBJ)
	@mkdir -p $(@D); rm -f $@; ar rcs $@ $^
$(OUT)/libEncoderLib.a: $(ENC_OBJ)
	@mkdir -p $(@D); rm -f $@; ar rcs $@ $^
$(OUT)/libUtilities.a: $(UTIL_OBJ)
	@mkdir -p $(@D); rm -f $@; ar rcs $@ $^

$(OUT)/DecoderApp: $(DECAPP_OBJ) $(OUT)/libDecoderLib.a $(OUT)/libCommonLib.a $(OUT)/libUtilities.a
	$(CXX) -pthread -o $@ $(DECAPP_OBJ) $(OUT)/libDecoderLib.a $(OUT)/libUtilities.a $(OUT)/libCommonLib.a
$(OUT)/EncoderApp: $(ENCAPP_OBJ) $(OUT)/libEncoderLib.a $(OUT)/libDecoderLib.a $(OUT)/libCommonLib.a $(OUT)/libUtilities.a
	$(CXX) -pthread -o $@ $(ENCAPP_OBJ) $(OUT)/libEncoderLib.a $(OUT)/libDecoderLib.a $(OUT)/libUtilities.a $(OUT)/libCommonLib.a

# capture tool: decodes with the reference DecLib and dumps descriptors + per-stage golden planes.
# The DecoderLib/CommonLib objects are linked as objects (not archives) so --wrap sees every call site.
CAP_SRC = $(CURDIR)/oracle/capture/vtm_capture.cpp
$(OUT)/obj/capture/vtm_capture.o: $(CAP_SRC) $(CURDIR)/oracle/capture/wraps.txt
	@mkdir -p $(@D); $(CXX) $(CXXFLAGS) -I$(SRC)/App/DecoderApp -c $< -o $@
CAPAPP_OBJ = $(call obj,$(SRC)/App/DecoderApp/DecApp.cpp $(SRC)/App/DecoderApp/DecAppCfg.cpp)
$(OUT)/vtm_capture: $(OUT)/obj/capture/vtm_capture.o $(CAPAPP_OBJ) $(DEC_OBJ) $(COMMON_OBJ) $(UTIL_OBJ) $(CURDIR)/oracle/capture/wraps.txt
	$(CXX) -pthread -o $@ $(OUT)/obj/capture/vtm_capture.o $(CAPAPP_OBJ) $(DEC_OBJ) $(UTIL_OBJ) $(COMMON_OBJ) $(WRAPFLAGS)

# drop-in demonstration: the same source built with -DVVCR_DROPIN — DecApp / DecLib of
# the reference, unchanged, linked against libvvcr.so; every decoded picture comes from libvvcr
dropin: $(OUT)/vtm_vvcr
$(OUT)/obj/capture/vtm_vvcr.o: $(CAP_SRC) $(CURDIR)/oracle/capture/wraps.txt $(CURDIR)/include/vvcr.h
	@mkdir -p $(@D); $(CXX) $(CXXFLAGS) -DVVCR_DROPIN -I$(CURDIR)/include -I$(SRC)/App/DecoderApp -c $< -o $@
$(OUT)/vtm_vvcr: $(OUT)/obj/capture/vtm_vvcr.o $(CAPAPP_OBJ) $(DEC_OBJ) $(COMMON_OBJ) $(UTIL_OBJ) $(CURDIR)/vvc_amd/libvvcr.so
	$(CXX) -pthread -o $@ $(OUT)/obj/capture/vtm_vvcr.o $(CAPAPP_OBJ) $(DEC_OBJ) $(UTIL_OBJ) $(COMMON_OBJ) $(WRAPFLAGS) \
	  -L$(CURDIR)/vvc_amd -lvvcr -Wl,-rpath,'$$ORIGIN/../../vvc_amd' -Wl,-rpath-link,/opt/rocm/lib

# EncoderApp drop-in: the reference EncoderApp / EncoderLib, unchanged, linked against
# libvvcr.so; the merge pass's Hadamard SATD goes through vvcr_rd_dist (oracle/capture/enc_vvcr.cpp).
# -rdynamic: the binding resolves the call site of RdCost::setDistParam with dladdr.
ENC_WRAP = -Wl,--wrap=_ZN6RdCost12setDistParamER9DistParamRK7AreaBufIKsES6_i11ComponentIDb
encdropin: $(OUT)/vtm_enc_vvcr
$(OUT)/obj/capture/enc_vvcr.o: $(CURDIR)/oracle/capture/enc_vvcr.cpp $(CURDIR)/include/vvcr.h
	@mkdir -p $(@D); $(CXX) $(CXXFLAGS) -I$(CURDIR)/include -c $< -o $@
$(OUT)/vtm_enc_vvcr: $(OUT)/obj/capture/enc_vvcr.o $(ENCAPP_OBJ) $(OUT)/libEncoderLib.a $(OUT)/libDecoderLib.a $(OUT)/libCommonLib.a $(OUT)/libUtilities.a $(CURDIR)/vvc_amd/libvvcr.so
	$(CXX) -pthread -rdynamic -o $@ $(OUT)/obj/capture/enc_vvcr.o $(ENCAPP_OBJ) $(OUT)/libEncoderLib.a $(OUT)/libDecoderLib.a \
	  $(OUT)/libUtilities.a $(OUT)/libCommonLib.a $(ENC_WRAP) -ldl \
	  -L$(CURDIR)/vvc_amd -lvvcr -Wl,-rpath,'$$ORIGIN/../../vvc_amd' -Wl,-rpath-link,/opt/rocm/lib

# RDO known-answer harness (RdCost distortion + forward transforms of the reference, oracle/capture/rdo_kat.cpp)
rdo_kat: $(OUT)/rdo_kat
$(OUT)/obj/capture/rdo_kat.o: $(CURDIR)/oracle/capture/rdo_kat.cpp
	@mkdir -p $(@D); $(CXX) $(CXXFLAGS) -c $< -o $@
$(OUT)/rdo_kat: $(OUT)/obj/capture/rdo_kat.o $(OUT)/libCommonLib.a
	$(CXX) -pthread -o $@ $(OUT)/obj/capture/rdo_kat.o $(OUT)/libCommonLib.a

# MC known-answer harness (InterpolationFilter::filterHor / filterVer of the reference, oracle/capture/mc_kat.cpp)
mc_kat: $(OUT)/mc_kat
$(OUT)/obj/capture/mc_kat.o: $(CURDIR)/oracle/capture/mc_kat.cpp
	@mkdir -p $(@D); $(CXX) $(CXXFLAGS) -c $< -o $@
$(OUT)/mc_kat: $(OUT)/obj/capture/mc_kat.o $(OUT)/libCommonLib.a
	$(CXX) -pthread -o $@ $(OUT)/obj/capture/mc_kat.o $(OUT)/libCommonLib.a

$(OUT)/obj/Lib/CommonLib/x86/sse41/%.o: $(SRC)/Lib/CommonLib/x86/sse41/%.cpp
	@mkdir -p $(@D); $(CXX) $(CXXFLAGS) -msse4.1 -DUSE_SSE41 -c $< -o $@
$(OUT)/obj/Lib/CommonLib/x86/sse42/%.o: $(SRC)/Lib/CommonLib/x86/sse42/%.cpp
	@mkdir -p $(@D); $(CXX) $(CXXFLAGS) -msse4.2 -DUSE_SSE42 -c $< -o $@
$(OUT)/obj/Lib/CommonLib/x86/avx/%.o: $(SRC)/Lib/CommonLib/x86/avx/%.cpp
	@mkdir -p $(@D); $(CXX) $(CXXFLAGS) -mavx -DUSE_AVX -c $< -o $@
$(OUT)/obj/Lib/CommonLib/x86/avx2/%.o: $(SRC)/Lib/CommonLib/x86/avx2/%.cpp
	@mkdir -p $(@D); $(CXX) $(CXXFLAGS) -mavx2 -DUSE_AVX2 -c $< -o $@
$(OUT)/obj/%.o: $(SRC)/%.cpp
	@mkdir -p $(@D); $(CXX) $(CXXFLAGS) -c $< -o $@

clean:
	rm -rf $(OUT)

.PHONY: all apps capture dropin encdropin clean
