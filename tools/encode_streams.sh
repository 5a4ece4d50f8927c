#!/bin/bash
# Re-creates the committed test bitstreams with the REFERENCE encoder built by oracle/ref.mk
# (VTM 7.3 EncoderApp, CTC configs from /root/reference/cfg). Test-infrastructure only; runs in the
# build container (needs /root/reference). Every stream carries MD5 decoded-picture-hash SEI.
#   tools/encode_streams.sh <name> ...     names: ai416_q37 ra416_q32 ai480_q32 ra480_q32 ra1080_q32 ra1080t_q32 ra2160_q27 ra2160_q32 ralm416_q32 ailm416_q37 rawp416_q32 ratile416_q32 ratile1080_q32 ra4320t_q32 ra1080l_q32 ra412c_q32 ra2160l_q27 ra2160l_q32 ra2160n_q27 rageo480_q32 aibdpcm416_q32 radq0416_q32 rawp1080_q32 ralmgeo416_q32 rawpp416_q32 rawpp1080_q32 ratilenf416_q32 ratilenf1080_q32 rasub480_q32 ravb416_q32 ravb416b_q37 raladf416_q32 rarsc416_q32
set -e
R=/root/reference/cfg; E=${E:-$(dirname $0)/../oracle/_ref/EncoderApp}; T=${T:-/tmp/enc}; O=${O:-$(dirname $0)/../tests/golden/streams}
mkdir -p $T $O
G="python3 $(dirname $0)/gen_synth.py"
TILES="--EnablePicPartitioning=1 --RasterScanSlices=1 --RasterSliceSizes=1000 --DisableLoopFilterAcrossTiles=0 --DisableLoopFilterAcrossSlices=0"
# tiles and raster-scan slices with the loop filters NOT across their boundaries (LoopFilter.cpp:670,920;
# SampleAdaptiveOffset.cpp:692; AdaptiveLoopFilter.cpp:129): each slice one row of tiles
TILESNF="--EnablePicPartitioning=1 --RasterScanSlices=1 --DisableLoopFilterAcrossTiles=1 --DisableLoopFilterAcrossSlices=1"
EFAST="--SearchRange=64 --LCTUFast=1 --FastMrg=1 --PBIntraFast=1 --FastMIP=1 --FastLFNST=1 --ISPFast=1 --BcwFast=1 --TransformSkipFast=1"
FAST="--SearchRange=32 --MaxMTTHierarchyDepth=1 --MaxMTTHierarchyDepthISliceL=1 --MaxMTTHierarchyDepthISliceC=1 --LCTUFast=1 --FastMrg=1 --PBIntraFast=1 --FastMIP=1 --FastLFNST=1 --ISPFast=1 --BcwFast=1 --TransformSkipFast=1"
enc() { # name cfg W H frames qp yuv extra...
  local n=$1 cfg=$2 w=$3 h=$4 f=$5 q=$6 y=$7; shift 7
  $E -c $R/$cfg -i $y -wdt $w -hgt $h -fr 50 -f $f -q $q --InputBitDepth=8 --SEIDecodedPictureHash=1 \
     -b $O/$n.bin -o /dev/null "$@" > $T/enc_$n.log
}
for n in "$@"; do case $n in
  ai416_q37)  [ -f $T/syn416.yuv ]  || $G 416 240 17 $T/syn416.yuv;   enc $n encoder_intra_vtm.cfg 416 240 8 37 $T/syn416.yuv --TemporalSubsampleRatio=1 ;;
  ra416_q32)  [ -f $T/syn416.yuv ]  || $G 416 240 17 $T/syn416.yuv;   enc $n encoder_randomaccess_vtm.cfg 416 240 17 32 $T/syn416.yuv ;;
  ai480_q32)  [ -f $T/syn480.yuv ]  || $G 832 480 33 $T/syn480.yuv;   enc $n encoder_intra_vtm.cfg 832 480 8 32 $T/syn480.yuv --TemporalSubsampleRatio=1 ;;
  ra480_q32)  [ -f $T/syn480.yuv ]  || $G 832 480 33 $T/syn480.yuv;   enc $n encoder_randomaccess_vtm.cfg 832 480 33 32 $T/syn480.yuv --SearchRange=64 ;;
  ra1080_q32) [ -f $T/syn1080.yuv ] || $G 1920 1080 9 $T/syn1080.yuv; enc $n encoder_randomaccess_vtm.cfg 1920 1080 9 32 $T/syn1080.yuv --SearchRange=64 ;;
  # 33 pictures: a whole intra period of the CTC random-access configuration (IntraPeriod 32, GOP 16)
  ra1080l_q32) [ -f $T/syn1080l.yuv ] || $G 1920 1080 33 $T/syn1080l.yuv; enc $n encoder_randomaccess_vtm.cfg 1920 1080 33 32 $T/syn1080l.yuv --SearchRange=64 ;;
  ra1080t_q32) [ -f $T/syn1080t.yuv ] || $G 1920 1080 9 $T/syn1080t.yuv 0; enc $n encoder_randomaccess_vtm.cfg 1920 1080 9 32 $T/syn1080t.yuv --SearchRange=64 ;;
  ra2160_q27) [ -f $T/syn2160.yuv ] || $G 3840 2160 3 $T/syn2160.yuv; enc $n encoder_randomaccess_vtm.cfg 3840 2160 3 27 $T/syn2160.yuv --SearchRange=64 ;;
  ra2160_q32) [ -f $T/syn2160.yuv ] || $G 3840 2160 3 $T/syn2160.yuv; enc $n encoder_randomaccess_vtm.cfg 3840 2160 3 32 $T/syn2160.yuv --SearchRange=64 ;;
  # video-range content: the reference encoder keeps LMCS (luma mapping + chroma residual scaling) on
  ralm416_q32) [ -f $T/syn416v.yuv ] || $G 416 240 17 $T/syn416v.yuv 0.002 1; enc $n encoder_randomaccess_vtm.cfg 416 240 17 32 $T/syn416v.yuv ;;
  # brightness fade with explicit weighted prediction on (WeightPrediction::xWeightedPredictionBi/Uni)
  rawp416_q32) [ -f $T/syn416f.yuv ] || $G 416 240 17 $T/syn416f.yuv 0.002 0 0.03; enc $n encoder_randomaccess_vtm.cfg 416 240 17 32 $T/syn416f.yuv --WeightedPredP=1 --WeightedPredB=1 ;;
  ailm416_q37) [ -f $T/syn416v.yuv ] || $G 416 240 17 $T/syn416v.yuv 0.002 1; enc $n encoder_intra_vtm.cfg 416 240 8 37 $T/syn416v.yuv --TemporalSubsampleRatio=1 ;;
  # tile rows (one raster-scan slice holding every tile; loop filters cross tile edges): the spatial
  # shards of the multi-GPU path -- intra / CABAC stop at tile rows, DBK/SAO/ALF do not
  ratile416_q32) [ -f $T/syn416.yuv ] || $G 416 240 17 $T/syn416.yuv; enc $n encoder_randomaccess_vtm.cfg 416 240 17 32 $T/syn416.yuv $TILES --TileColumnWidthArray=4 --TileRowHeightArray=1 ;;
  ratile1080_q32) [ -f $T/syn1080.yuv ] || $G 1920 1080 9 $T/syn1080.yuv; enc $n encoder_randomaccess_vtm.cfg 1920 1080 9 32 $T/syn1080.yuv --SearchRange=64 $TILES --TileColumnWidthArray=15 --TileRowHeightArray=1 ;;
  # 8K, 8 tile rows (4,4,4,4,4,4,5,5 CTU rows); encoder fast-search settings only (the coded tools are the CTC set)
  ra4320t_q32) [ -f $T/syn4320.yuv ] || $G 7680 4320 3 $T/syn4320.yuv; enc $n encoder_randomaccess_vtm.cfg 7680 4320 3 32 $T/syn4320.yuv $TILES $FAST --TileColumnWidthArray=60 --TileRowHeightArray="4 4 4 4 4 4 5" ;;
  # 412x236 coded as 416x240 with a conformance window (the encoder pads right / bottom to the 8-sample
  # minimum CU size): DecoderApp's output crops it (VideoIOYuv::write), vvcr_write_output must too
  ra412c_q32) [ -f $T/syn412.yuv ] || $G 412 236 5 $T/syn412.yuv; enc $n encoder_randomaccess_vtm.cfg 412 236 5 32 $T/syn412.yuv --ConformanceWindowMode=1 ;;
  # 4K random access, a whole GOP-16 after the intra picture (17 pictures), so the I picture is 1/17 of
  # the work as in the CTC random-access configuration (BASELINE configs[2] QP27, north star QP32).
  # Encoder-side speed-ups only (search range, fast decisions, multi-type-tree search depth 1 as for 8K:
  # the CTC-depth search took ~90 min per 4K picture here); the coded tool set is the CTC one.
  # ra2160n: the first 9 pictures (I + the first 8 of the GOP), a shorter run of the same encode.
  ra2160l_q27) [ -f $T/syn2160l.yuv ] || $G 3840 2160 17 $T/syn2160l.yuv; enc $n encoder_randomaccess_vtm.cfg 3840 2160 17 27 $T/syn2160l.yuv $FAST ;;
  ra2160l_q32) [ -f $T/syn2160l.yuv ] || $G 3840 2160 17 $T/syn2160l.yuv; enc $n encoder_randomaccess_vtm.cfg 3840 2160 17 32 $T/syn2160l.yuv $FAST ;;
  ra2160n_q27) [ -f $T/syn2160l.yuv ] || $G 3840 2160 17 $T/syn2160l.yuv; enc $n encoder_randomaccess_vtm.cfg 3840 2160 9 27 $T/syn2160l.yuv $FAST ;;
  # a second independently moving layer cut by polygon edges: GEO (InterPrediction.cpp:1749) and CIIP
  # (IntraPrediction.cpp:681,735) CUs in quantity
  rageo480_q32) [ -f $T/syn480g.yuv ] || $G 832 480 17 $T/syn480g.yuv 0.002 0 0 layers; enc $n encoder_randomaccess_vtm.cfg 832 480 17 32 $T/syn480g.yuv ;;
  # screen-like content, BDPCM (luma; VTM 7.3 allows chroma BDPCM only in 4:4:4, VLCWriter.cpp:965) (IntraPrediction.cpp:644, TrQuant.cpp:533)
  aibdpcm416_q32) [ -f $T/syn416s.yuv ] || $G 416 240 17 $T/syn416s.yuv 0 0 0 screen; enc $n encoder_intra_vtm.cfg 416 240 8 32 $T/syn416s.yuv --TemporalSubsampleRatio=1 --BDPCM=1 ;;
  # scalar dequantisation on every block (Quant.cpp:369), sign data hiding, explicit MTS for inter too
  radq0416_q32) [ -f $T/syn416g.yuv ] || $G 416 240 17 $T/syn416g.yuv 0.002 0 0 layers; enc $n encoder_randomaccess_vtm.cfg 416 240 17 32 $T/syn416g.yuv --DepQuant=0 --SignHideFlag=1 --MTS=3 ;;
  # the layered GEO / CIIP content in video range, so LMCS stays on: CIIP CUs in LMCS inter slices (the
  # forward-mapped inter prediction blended with the intra one, IntraPrediction.cpp:681, DecCu.cpp:719)
  ralmgeo416_q32) [ -f $T/syn416gv.yuv ] || $G 416 240 17 $T/syn416gv.yuv 0.002 1 0 layers; enc $n encoder_randomaccess_vtm.cfg 416 240 17 32 $T/syn416gv.yuv ;;
  # explicit weighted prediction at 1080p (WeightPrediction.cpp:382,413)
  rawp1080_q32) [ -f $T/syn1080f.yuv ] || $G 1920 1080 9 $T/syn1080f.yuv 0.002 0 0.03; enc $n encoder_randomaccess_vtm.cfg 1920 1080 9 32 $T/syn1080f.yuv --SearchRange=64 --WeightedPredP=1 --WeightedPredB=1 ;;
  # wavefront parallel processing (entropy coding sync: DecSlice.cpp:160-176, one substream per CTU row)
  rawpp416_q32) [ -f $T/syn416.yuv ] || $G 416 240 17 $T/syn416.yuv; enc $n encoder_randomaccess_vtm.cfg 416 240 17 32 $T/syn416.yuv --WaveFrontSynchro=1 ;;
  rawpp1080_q32) [ -f $T/syn1080.yuv ] || $G 1920 1080 9 $T/syn1080.yuv; enc $n encoder_randomaccess_vtm.cfg 1920 1080 9 32 $T/syn1080.yuv $FAST --WaveFrontSynchro=1 ;;
  # 2 x 2 tiles (2 CTU columns, 1 CTU row each), two raster slices of 2 tiles, no loop filtering across either
  # BASELINE config 4's subpicture layout at the size its reference cfg is written for: 2 subpictures, 4
  # explicit rectangular slices (one tile each), loop filters not across tiles / slices (9 pictures)
  rasub480_q32) [ -f $T/syn480s.yuv ] || $G 832 480 17 $T/syn480s.yuv; enc $n encoder_randomaccess_vtm.cfg 832 480 9 32 $T/syn480s.yuv -c $R/nonCTC-SliceConfigExamples/subpicture_4Slice2VerSubPic.cfg --SearchRange=64 ;;
  # virtual boundaries, loop filters not across them (one vertical at x = 192, one horizontal at y = 96, both
  # inside 128 x 128 CTUs): deblocking edges dropped, SAO / ALF per sub-rectangle (9 pictures)
  ravb416_q32) [ -f $T/syn416.yuv ] || $G 416 240 17 $T/syn416.yuv; enc $n encoder_randomaccess_vtm.cfg 416 240 9 32 $T/syn416.yuv --LoopFilterAcrossVirtualBoundariesDisabledFlag=1 --NumVerVirtualBoundaries=1 --VirtualBoundariesPosX=192 --NumHorVirtualBoundaries=1 --VirtualBoundariesPosY=96 ;;
  # two vertical boundaries (x = 128 on a CTU edge, x = 264 inside a CTU) and one horizontal on the CTU-row
  # edge (y = 128, where ALF's own CTU-row virtual boundary rows meet it), QP 37 (9 pictures)
  ravb416b_q37) [ -f $T/syn416.yuv ] || $G 416 240 17 $T/syn416.yuv; enc $n encoder_randomaccess_vtm.cfg 416 240 9 37 $T/syn416.yuv --LoopFilterAcrossVirtualBoundariesDisabledFlag=1 --NumVerVirtualBoundaries=2 --VirtualBoundariesPosX="128 264" --NumHorVirtualBoundaries=1 --VirtualBoundariesPosY=128 ;;
  # luma-adaptive deblocking (LADF: the encoder's default 3 intervals, QP offsets by the edge's mean luma)
  raladf416_q32) [ -f $T/syn416.yuv ] || $G 416 240 17 $T/syn416.yuv; enc $n encoder_randomaccess_vtm.cfg 416 240 9 32 $T/syn416.yuv --LADF=1 ;;
  # raster slices that start and end inside rows of 64x64 CTUs (1-CTU tiles, slices of 1 then 8 tiles), loop
  # filters across tiles but not across slices: SAO's diagonal neighbours and ALF's raster-slice corner
  # padding (AdaptiveLoopFilter.cpp:172-198) on the CTBs whose top-left / bottom-right neighbour is another slice
  rarsc416_q32) [ -f $T/syn416.yuv ] || $G 416 240 17 $T/syn416.yuv; enc $n encoder_randomaccess_vtm.cfg 416 240 9 32 $T/syn416.yuv --CTUSize=64 --EnablePicPartitioning=1 --TileColumnWidthArray=1 --TileRowHeightArray=1 --RasterScanSlices=1 --RasterSliceSizes="1 8" --DisableLoopFilterAcrossTiles=0 --DisableLoopFilterAcrossSlices=1 ;;
  ratilenf416_q32) [ -f $T/syn416.yuv ] || $G 416 240 17 $T/syn416.yuv; enc $n encoder_randomaccess_vtm.cfg 416 240 17 32 $T/syn416.yuv $TILESNF --TileColumnWidthArray=2 --TileRowHeightArray=1 --RasterSliceSizes=2 ;;
  # 3 x 3 tiles of 5 x 3 CTUs, a raster slice per tile row, no loop filtering across tiles or slices
  ratilenf1080_q32) [ -f $T/syn1080.yuv ] || $G 1920 1080 9 $T/syn1080.yuv; enc $n encoder_randomaccess_vtm.cfg 1920 1080 9 32 $T/syn1080.yuv $FAST $TILESNF --TileColumnWidthArray=5 --TileRowHeightArray=3 --RasterSliceSizes=3 ;;
  *) echo "unknown stream $n"; exit 1 ;;
esac; done
