#!/bin/bash
# Re-creates the committed test bitstreams with the REFERENCE encoder built by oracle/ref.mk
# (VTM 7.3 EncoderApp, CTC configs from /root/reference/cfg). Test-infrastructure only; runs in the
# build container (needs /root/reference). Every stream carries MD5 decoded-picture-hash SEI.
#   tools/encode_streams.sh <name> ...     names: ai416_q37 ra416_q32 ai480_q32 ra480_q32 ra1080_q32 ra1080t_q32 ra2160_q27 ra2160_q32 ralm416_q32 ailm416_q37 rawp416_q32
set -e
R=/root/reference/cfg; E=${E:-$(dirname $0)/../oracle/_ref/EncoderApp}; T=${T:-/tmp/enc}; O=${O:-$(dirname $0)/../tests/golden/streams}
mkdir -p $T $O
G="python3 $(dirname $0)/gen_synth.py"
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
  ra1080t_q32) [ -f $T/syn1080t.yuv ] || $G 1920 1080 9 $T/syn1080t.yuv 0; enc $n encoder_randomaccess_vtm.cfg 1920 1080 9 32 $T/syn1080t.yuv --SearchRange=64 ;;
  ra2160_q27) [ -f $T/syn2160.yuv ] || $G 3840 2160 3 $T/syn2160.yuv; enc $n encoder_randomaccess_vtm.cfg 3840 2160 3 27 $T/syn2160.yuv --SearchRange=64 ;;
  ra2160_q32) [ -f $T/syn2160.yuv ] || $G 3840 2160 3 $T/syn2160.yuv; enc $n encoder_randomaccess_vtm.cfg 3840 2160 3 32 $T/syn2160.yuv --SearchRange=64 ;;
  # video-range content: the reference encoder keeps LMCS (luma mapping + chroma residual scaling) on
  ralm416_q32) [ -f $T/syn416v.yuv ] || $G 416 240 17 $T/syn416v.yuv 0.002 1; enc $n encoder_randomaccess_vtm.cfg 416 240 17 32 $T/syn416v.yuv ;;
  # brightness fade with explicit weighted prediction on (WeightPrediction::xWeightedPredictionBi/Uni)
  rawp416_q32) [ -f $T/syn416f.yuv ] || $G 416 240 17 $T/syn416f.yuv 0.002 0 0.03; enc $n encoder_randomaccess_vtm.cfg 416 240 17 32 $T/syn416f.yuv --WeightedPredP=1 --WeightedPredB=1 ;;
  ailm416_q37) [ -f $T/syn416v.yuv ] || $G 416 240 17 $T/syn416v.yuv 0.002 1; enc $n encoder_intra_vtm.cfg 416 240 8 37 $T/syn416v.yuv --TemporalSubsampleRatio=1 ;;
  *) echo "unknown stream $n"; exit 1 ;;
esac; done
