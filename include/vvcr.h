/*
 * vvcr.h — C-ABI of libvvcr, the MI355X (gfx950) VVC decode-reconstruction path.
 *
 * Drop-in boundary for VTM 7.3 (ultrawide/vvc). The reference reconstructs per block through C
 * function-pointer tables (InterpolationFilter::m_filterHor/m_filterVer/m_filterCopy
 * source/Lib/CommonLib/InterpolationFilter.h:100-107, PelBufferOps g_pelBufOP Buffer.h:54-88,
 * fastInvTrans TrQuant.cpp:69-81, AdaptiveLoopFilter::m_filter5x5Blk/m_filter7x7Blk
 * AdaptiveLoopFilter.h:101-133) called from DecCu::decompressCtu (DecoderLib/DecCu.cpp:102), once per
 * CTU from DecSlice::decompressSlice (DecSlice.cpp:204), and through the picture-level loop filters in
 * DecLib::executeLoopFilters (DecLib.cpp:560-623). libvvcr replaces both at PICTURE granularity:
 *
 *   DecSlice::decompressSlice (last slice of a picture)  ->  vvcr_begin_picture + vvcr_submit
 *   DecLib::executeLoopFilters                           ->  vvcr_end_picture (recon + DBK + SAO + ALF)
 *   CS::setRefinedMotionField (UnitTools.cpp:68)          <-  vvcr_get_dmvr_deltas
 *   DecApp::xWriteOutput / DecLib::finishPicture MD5      <-  vvcr_read_picture
 *
 * Descriptor rows (vvcr_cu / vvcr_pu / vvcr_tu) are the parsed, MV-derived coding units of one
 * picture in decode order, i.e. the contents of CodingStructure::cus/pus/tus (CodingStructure.h:194-196)
 * after DecCu::xDeriveCUMV (DecCu.cpp:878); field meaning follows CodingUnit / PredictionUnit /
 * TransformUnit (Unit.h:288-456). All fields are int32 so a row is a plain array.
 *
 * Conventions: every entry point returns 0 on success or a negative VVCR_E_* code; no C++
 * exception crosses the ABI; vvcr_last_error() gives the message. The library owns all device
 * memory (DPB slots, scratch); the caller owns host arrays until the call returns (deep copy).
 * Samples are 10-bit in uint16/int16 ("Pel", TypeDef.h:313), 4:2:0.
 */
#ifndef VVCR_H
#define VVCR_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VVCR_OK 0
#define VVCR_E_ARG -1
#define VVCR_E_HIP -2
#define VVCR_E_STATE -3
#define VVCR_E_UNSUPPORTED -4
#define VVCR_MAX_REF 16
#define VVCR_MAX_TILE_LINES 64   /* tile columns / rows per picture */

typedef struct vvcr_ctx vvcr_ctx;

/* Sequence-level parameters (SPS subset, Slice.h SPS): replaces Picture::create / PelStorage::create
 * (Picture.cpp:195-214, Buffer.cpp:687) — the DPB lives in HBM, without border margins (MC clamps
 * coordinates instead of Picture::extendPicBorder, Picture.cpp:737). */
typedef struct vvcr_seq_params {
  int32_t width, height;       /* luma samples */
  int32_t chroma_format;       /* 1 = 4:2:0 (only supported format) */
  int32_t bit_depth;           /* luma = chroma bit depth (8..10) */
  int32_t ctu_log2;            /* 5..7 */
  int32_t dpb_slots;           /* number of picture buffers to allocate (1..256) */
  int32_t device;              /* HIP device ordinal */
} vvcr_seq_params;

/* CodingUnit (Unit.h:288-372). x,y,w,h = luma area (CU::lumaPos/lumaSize); cx..ch = Cb area. */
typedef struct vvcr_cu {
  int32_t x, y, w, h, cx, cy, cw, ch;
  int32_t chtype, predmode, qp, treetype, modetype, skip, mmvdskip, affine, affinetype, geo;
  int32_t bdpcm, bdpcmc, imv, rootcbf, sbtinfo, mtsflag, lfnst, bcw, mip, isp;
  int32_t smvd, act, cqpadj, depth, qtdepth, firstpu, npu, firsttu, ntu, slice;
  int32_t yvalid, cvalid;
} vvcr_cu;

/* PredictionUnit (Unit.h:378-456). mv in 1/16 luma sample (MV_FRACTIONAL_BITS_INTERNAL=4,
 * CommonDef.h:281), already derived (merge / AMVP / MMVD / SMVD resolved). ref0/ref1 = refIdx.
 * aff[l*6 + k*2 + {0,1}] = mvAffi[l][k]. fidir_l / fidir_c = PU::getFinalIntraMode.
 * bdof / dmvr = the producer's evaluation of the reference conditions
 * (InterPrediction.cpp:1584-1635, UnitTools.cpp:1249 PU::checkDMVRCondition). */
typedef struct vvcr_pu {
  int32_t cu, x, y, w, h, cx, cy, cw, ch, chtype;
  int32_t idir_l, idir_c, fidir_l, fidir_c, mipt, mrl;
  int32_t merge, regmerge, mergeidx, geodir, geoi0, geoi1, mmvd, interdir;
  int32_t mv0x, mv0y, mv1x, mv1y, ref0, ref1, mrgtype, mvrefine, ciip;
  int32_t aff[12];
  int32_t dmvr_off, bdof, dmvr;
} vvcr_pu;

/* TransformUnit (Unit.h:458+). Per component c: b[c] = {x, y, w, h, cbf, mts, coef_off, qp, qp_ts}.
 * coef_off indexes the coefficient pool (TCoeff levels, w*h row-major, as parsed:
 * TransformUnit::getCoeffs); qp / qp_ts = QpParam::Qp(false/true) (Quant.h:68-102). */
typedef struct vvcr_tu {
  int32_t cu, chtype, depth, noresi, jccr, cadj;
  int32_t b[3][9];
} vvcr_tu;

/* Per-4x4 motion field (MotionInfo, MotionInfo.h:101), before DMVR write-back: what deblocking
 * boundary strength and sub-block (SbTMVP) motion compensation read. */
typedef struct vvcr_motion {
  int32_t is_inter, inter_dir, ref0, ref1, mv0x, mv0y, mv1x, mv1y, bcw, alt_hpel;
} vvcr_motion;

/* GEO candidate pair captured at InterPrediction::motionCompensationGeo (InterPrediction.cpp:1749). */
typedef struct vvcr_geo {
  int32_t cu;
  int32_t cand[2][6];          /* inter_dir, list, ref_idx, mvx, mvy, alt_hpel */
} vvcr_geo;

/* SAO per CTB and component (SAOOffset, TypeDef.h:938) after SampleAdaptiveOffset::
 * reconstructBlkSAOParam (SampleAdaptiveOffset.cpp:231): merges resolved, offsets de-quantised.
 * mode: 0 off / 1 new / 2 merge(resolved); type: 0..3 EO_0/90/135/45, 4 BO; offset[32] indexed by
 * band (BO) or edge class 0..4 (EO). */
typedef struct vvcr_sao {
  int32_t mode, type, band, offset[32];
} vvcr_sao;

/* Picture-level parameters (slice / picture header subset). */
typedef struct vvcr_pic_params {
  int32_t poc, slot, slice_type, slice_qp;
  int32_t num_ref[2];
  int32_t ref_slot[2][VVCR_MAX_REF];
  int32_t ref_poc[2][VVCR_MAX_REF];
  int32_t ref_lt[2][VVCR_MAX_REF];
  int32_t dual_tree, dep_quant, sign_hiding, joint_cbcr;
  int32_t bdof_enabled, dmvr_enabled, prof_enabled, lfnst_enabled, mts_intra, mts_inter, sbt;
  int32_t wp_p, wp_b;
  int32_t wp[2][VVCR_MAX_REF][3][7];  /* present, log2denom, weight, offset, w, o, offset(scaled) */
  int32_t dbk_disable, dbk_beta_offset_div2, dbk_tc_offset_div2;
  int32_t lf_across_slices, lf_across_tiles;
  int32_t chroma_qp_off[3];          /* pps + slice chroma QP offsets: [1] Cb, [2] Cr, [0] joint Cb-Cr */
  int32_t chroma_qp_map[3][128];     /* SPS::getMappedChromaQpValue for qp in [-64,63] at [c][qp+64];
                                        [0] = JOINT_CbCr table (QpParam, Quant.cpp:121) */
  int32_t sao_luma, sao_chroma;
  int32_t alf_en[3], ccalf_en[2], alf_vb_luma, alf_vb_chroma;
  int32_t lmcs_enabled, lmcs_chroma_scale, lmcs_min_bin, lmcs_max_bin;
  int16_t lmcs_fwd[1024], lmcs_inv[1024], lmcs_pivot[17];
  int32_t lmcs_cadj[16];
  int32_t max_tb_log2, log2_max_ts;
  int32_t use_mts, implicit_mts, joint_cbcr_sign;
  /* Tiles (PPS::getTileColumnBd / getTileRowBd, in CTUs; bd[n] = picture size in CTUs). num_tile_* = 0
   * means one tile. Intra prediction, CCLM, CIIP and LMCS chroma scaling read neighbours of the same
   * slice (vvcr_cu.slice) and tile only (CodingStructure::getCURestricted, CodingStructure.cpp:1519). */
  int32_t num_tile_cols, num_tile_rows;
  int32_t tile_col_bd[VVCR_MAX_TILE_LINES + 1], tile_row_bd[VVCR_MAX_TILE_LINES + 1];
  int32_t entropy_sync;        /* WPP (pps entropy_coding_sync): per-row contexts; intra reads no CU beyond the current CTU column */
  /* Spatial shard (multi-GPU): luma rows [shard_y0, shard_y1) of the picture, on tile-row
   * boundaries; shard_y1 = 0 means the whole picture. Reconstruction covers the CUs of the shard only.
   * The loop-filter stages then produce the final samples of the shard's rows and need, in the picture
   * slot, the reconstructed (pre-deblocking, post-LMCS-inverse) samples of the VVCR_LF_HALO luma rows
   * above and below the shard (the neighbours' rows: vvcr_import_rows) and the descriptors of the CUs
   * there (they are part of the submitted picture). Motion compensation reads reference rows within
   * the picture's reach (vvcr_picture_work_counts counts[8..9]); they must be present in the slots. */
  int32_t shard_y0, shard_y1;
  /* Virtual boundaries (ph / sps_loop_filter_across_virtual_boundaries_disabled_present_flag, luma samples,
   * multiples of 8): no deblocking edge on them, no SAO edge-offset sample next to them, ALF filters each
   * side as if the other were outside the picture (LoopFilter.cpp:410-452, SampleAdaptiveOffset.cpp:96-116,
   * 731-750, AdaptiveLoopFilter.cpp:79-120, 458-483). vb_disabled = 0: none. */
  int32_t vb_disabled, num_vb_ver, vb_ver[3], num_vb_hor, vb_hor[3];
  /* Luma-adaptive deblocking (sps_ladf_*, LoopFilter::deriveLADFShift LoopFilter.cpp:815-840, applied at
   * :938-943): a luma edge's QP gains ladf_qp_offset[k] of the last interval k whose lower bound the mean of
   * its p0 / q0 samples on lines 0 and 3 exceeds (ladf_lower_bound[0] = 0). ladf_num = 0: off. */
  int32_t ladf_num, ladf_qp_offset[5], ladf_lower_bound[5];
} vvcr_pic_params;

#define VVCR_LF_HALO 24   /* luma rows (chroma: 12) of pre-deblocking samples a shard's loop filters read */

/* ALF / CC-ALF filters of the picture (AdaptiveLoopFilter::reconstructCoeffAPSs result,
 * AdaptiveLoopFilter.cpp:620) and per-CTB control (Picture.h:265-297). */
typedef struct vvcr_alf {
  int32_t num_luma_sets;                 /* 16 fixed + slice APS sets */
  const int16_t *luma_coef;              /* [num_luma_sets][25][13] */
  const int16_t *luma_clip;              /* [num_luma_sets][25][13] clipping values */
  const int16_t *chroma_coef;            /* [8][7] */
  const int16_t *chroma_clip;            /* [8][7] */
  const int16_t *cc_coef;                /* [2][4][8] */
  const uint8_t *ctb_en;                 /* [3][n_ctb] */
  const uint8_t *ctb_alt;                /* [3][n_ctb] chroma alternative */
  const int16_t *ctb_filter_set;         /* [n_ctb] luma filter set index */
  const uint8_t *cc_ctl;                 /* [2][n_ctb] CC-ALF filter idx + 1, 0 = off */
} vvcr_alf;

int vvcr_create(const vvcr_seq_params *sp, vvcr_ctx **out);
int vvcr_destroy(vvcr_ctx *ctx);
/* Message of the last failing call MADE BY THE CALLING THREAD (like errno): with ctx the last failing
 * context call of this thread, whatever context it was on; with NULL the last failing vvcr_create of this
 * thread. Several threads may prepare pictures of one context at once, so the text is never shared
 * between threads; read it on the thread that saw the error code. */
const char *vvcr_last_error(vvcr_ctx *ctx);

int vvcr_begin_picture(vvcr_ctx *ctx, const vvcr_pic_params *pp);
/* Copies one picture's descriptors into pinned staging and uploads them asynchronously. */
int vvcr_submit(vvcr_ctx *ctx,
                const vvcr_cu *cu, int32_t ncu,
                const vvcr_pu *pu, int32_t npu,
                const vvcr_tu *tu, int32_t ntu,
                const int32_t *coef, int64_t ncoef,
                const vvcr_motion *motion,          /* (height/4) x (width/4) */
                const vvcr_geo *geo, int32_t ngeo);
int vvcr_set_loop_filter_params(vvcr_ctx *ctx, const vvcr_sao *sao /* [n_ctb][3] */, const vvcr_alf *alf);

/* Stage mask for vvcr_end_picture_stages (tests isolate stages; vvcr_end_picture runs all). */
#define VVCR_STAGE_RESID 0x01   /* dequant + inverse transform of every TU -> residual planes */
#define VVCR_STAGE_INTER 0x02   /* motion compensation (+ BDOF/DMVR/affine/GEO/CIIP) + inter recon */
#define VVCR_STAGE_INTRA 0x04   /* intra prediction dependency waves + recon */
#define VVCR_STAGE_LMCS_INV 0x08
#define VVCR_STAGE_DBK 0x10
#define VVCR_STAGE_SAO 0x20
#define VVCR_STAGE_ALF 0x40
#define VVCR_STAGE_ALL 0x7f
int vvcr_end_picture(vvcr_ctx *ctx);
int vvcr_end_picture_stages(vvcr_ctx *ctx, uint32_t stage_mask);

/* Two-phase form of vvcr_end_picture: prepare plans the picture on the host and uploads every input
 * (descriptors, work lists, loop-filter parameters) into device memory owned by the returned handle;
 * launch enqueues the picture's kernels (reading device-resident data only) and may be repeated, e.g.
 * to replay a resident sequence; release frees the handle after its last launch completed.
 *
 * Ordering: launches are asynchronous and run on one of the context's execution lanes (HIP streams with
 * their own scratch planes). A picture starts once the pictures it depends on through the DPB are done:
 * the last writer of each of its reference slots, and the last writer and all readers since of its own
 * slot. Pictures without such a dependency (e.g. the pictures of one temporal layer, or the intra
 * picture of the next segment) may run concurrently. Host reads/writes of planes, vvcr_sync and
 * vvcr_get_dmvr_deltas wait for the work they depend on. */
int vvcr_prepare_picture(vvcr_ctx *ctx, uint32_t stage_mask, int32_t *handle);
int vvcr_launch_picture(vvcr_ctx *ctx, int32_t handle);
/* Launches only the stages of stage_mask that the picture was prepared with, e.g. the reconstruction
 * stages and, after a halo exchange, the loop-filter stages of one prepared spatial shard (each launch
 * orders itself after the slot's earlier writer like any other). */
int vvcr_launch_picture_stages(vvcr_ctx *ctx, int32_t handle, uint32_t stage_mask);
/* Frame-batched launch of n (1..4) prepared inter pictures that do not reference each other and write
 * different slots (e.g. the adjacent top-temporal-layer pictures POC 1 / 3 of a GOP-16 hierarchy, which
 * DecApp decodes one after the other, with POC 6): one execution lane runs their residuals, ONE plain-MC launch for
 * all of them (a single 4K picture's k_mc is one partial round of waves), then each picture's remaining
 * stages. Equivalent to launching them one by one (VVCR_E_ARG when a picture references another of the
 * batch, shares its slot, or was prepared without every stage). vvcr_kernel_stat.pictures of the plain-MC
 * group tells which record holds the batched launch's time (pictures = n) and which were carried (0). */
int vvcr_launch_pictures(vvcr_ctx *ctx, const int32_t *handles, int32_t n);
int vvcr_release_picture(vvcr_ctx *ctx, int32_t handle);

/* Host-only picture builder: the same begin / submit / loop-filter / plan sequence on a standalone
 * object that needs no context and no device, so a parallel host producer (one thread per picture —
 * the reference decodes a picture's slices in DecLib::decode / DecSlice::decompressSlice, DecLib.cpp:1753)
 * can validate and plan several pictures at once. vvcr_prepare_planned then only uploads the planned
 * work lists into a prepared-picture handle of ctx; it may be called from several threads at once
 * (each with its own picture). pp->slot / ref_slot are checked against sp->dpb_slots.
 *   vvcr_picture_work_counts: counts[0..7] = transform blocks, MC blocks, DMVR/BDOF blocks, affine tiles,
 *   inter recon tiles, intra steps, deblocking segments, DMVR sub-blocks; counts[8..9] = the first and
 *   one past the last luma row of the reference pictures the motion compensation reads (0, 0 without
 *   inter blocks); returns 10. */
typedef struct vvcr_picture vvcr_picture;
int vvcr_picture_create(const vvcr_seq_params *sp, const vvcr_pic_params *pp, vvcr_picture **out);
int vvcr_picture_submit(vvcr_picture *pic,
                        const vvcr_cu *cu, int32_t ncu,
                        const vvcr_pu *pu, int32_t npu,
                        const vvcr_tu *tu, int32_t ntu,
                        const int32_t *coef, int64_t ncoef,
                        const vvcr_motion *motion,
                        const vvcr_geo *geo, int32_t ngeo);
int vvcr_picture_set_loop_filter_params(vvcr_picture *pic, const vvcr_sao *sao, const vvcr_alf *alf);
int vvcr_picture_plan(vvcr_picture *pic, uint32_t stage_mask);
int vvcr_picture_work_counts(const vvcr_picture *pic, int64_t *counts, int32_t n);
const char *vvcr_picture_last_error(const vvcr_picture *pic);
int vvcr_picture_destroy(vvcr_picture *pic);
int vvcr_prepare_planned(vvcr_ctx *ctx, const vvcr_picture *pic, int32_t *handle);

/* Halo exchange of a spatial shard: copy luma rows [y0, y0 + n) of DPB slot and the co-located chroma
 * rows [y0 / 2, (y0 + n) / 2) of Cb and Cr (y0, n even) to / from a packed DEVICE buffer of
 * vvcr_rows_bytes(ctx, n) bytes: n luma rows of `width` int16 samples, then the Cb rows, then the Cr
 * rows. Export waits for the slot's last writer; import waits for its writer and readers; both return
 * once the copy is complete, so the caller may hand the buffer to a collective (RCCL) right away and
 * later launches see the imported rows. */
int64_t vvcr_rows_bytes(const vvcr_ctx *ctx, int32_t n);
int vvcr_export_rows(vvcr_ctx *ctx, int32_t slot, int32_t y0, int32_t n, void *dev_dst);
int vvcr_import_rows(vvcr_ctx *ctx, int32_t slot, int32_t y0, int32_t n, const void *dev_src);
/* The same copies enqueued on the caller's HIP stream (hipStream_t) without a host synchronisation: the
 * export runs after the slot's last writer and before the slot's next writer; the import after the
 * stream's earlier work (e.g. the collective that received the rows) and before every later launch that
 * reads or writes the slot. A halo exchange over RCCL on that stream is then ordered on the device. */
int vvcr_export_rows_async(vvcr_ctx *ctx, int32_t slot, int32_t y0, int32_t n, void *dev_dst, void *stream);
int vvcr_import_rows_async(vvcr_ctx *ctx, int32_t slot, int32_t y0, int32_t n, const void *dev_src, void *stream);

/* Per-kernel-group statistics of the last launch of a picture (handle 0 = the last launched picture):
 * HIP-event time on the library stream, number of kernel launches in the group and the algorithmic
 * bytes (each logical input and output counted once, 2 bytes per sample). Returns the number of groups. */
typedef struct vvcr_kernel_stat {
  char name[16];
  int32_t launches;
  float ms;
  double alg_bytes;
  int32_t pictures;   /* pictures the group's launches carried (a frame-batched k_mc: n on the first, 0 on the others) */
  int32_t pad;
} vvcr_kernel_stat;
int vvcr_kernel_stats(vvcr_ctx *ctx, int32_t handle, vvcr_kernel_stat *out, int32_t n);
/* Per-kernel-group event timing of later launches on (default) or off; with it off, vvcr_kernel_stats
 * reports ms = 0 (each event record is a marker packet in the execution lane's queue). */
int vvcr_set_timing(vvcr_ctx *ctx, int32_t on);
int vvcr_sync(vvcr_ctx *ctx);

/* Buffers addressable by vvcr_read_plane / vvcr_write_plane (tests and output). */
#define VVCR_BUF_RECO 0   /* picture slot (the DPB) */
#define VVCR_BUF_PRED 1   /* prediction plane of the current picture (MC output, before LMCS) */
#define VVCR_BUF_RESI 2   /* residual plane of the current picture */
int vvcr_read_plane(vvcr_ctx *ctx, int32_t buf, int32_t slot, int32_t comp, int16_t *dst, int32_t dst_stride);
int vvcr_write_plane(vvcr_ctx *ctx, int32_t buf, int32_t slot, int32_t comp, const int16_t *src, int32_t src_stride);
int vvcr_read_picture(vvcr_ctx *ctx, int32_t slot, uint16_t *planes[3], const int32_t strides[3]);

/* Output frame of a DPB slot exactly as DecoderApp writes it to its -o file (VideoIOYuv::write,
 * Utilities/VideoIOYuv.cpp:964-1047, writePlane :456-700; called from DecApp::xWriteOutput DecApp.cpp:853):
 * bit-depth change of scalePlane (:69-104; file bit depth = -d, 0 = the internal one; a smaller depth
 * rounds, (v + 2^(s-1)) >> s, and clips to [0, 2^d - 1], or to the BT.709 range with clip_rec709), samples
 * as bytes for 8-bit files and 16-bit little-endian otherwise, the conformance window cropped out (offsets
 * in luma samples: conf_win_*_offset times SubWidthC / SubHeightC) with every row still `width` samples
 * long and the cropped area at its top-left, zero-filled to the right and below, as VTM 7.3 writes it.
 * Planes Y, Cb, Cr one after the other; vvcr_output_bytes gives the frame size. dst: host memory
 * (dst_on_device 0; returns when the copy is complete) or device memory (1; returns when written). The
 * conversion runs on the GPU after the slot's last writer. */
typedef struct vvcr_output_params {
  int32_t file_bit_depth;       /* DecoderApp -d (0: internal bit depth) */
  int32_t conf_left, conf_right, conf_top, conf_bottom;
  int32_t clip_rec709;          /* DecoderApp --ClipOutputVideoToRec709Range */
} vvcr_output_params;
int64_t vvcr_output_bytes(const vvcr_ctx *ctx, const vvcr_output_params *op);
int vvcr_write_output(vvcr_ctx *ctx, int32_t slot, const vvcr_output_params *op, void *dst, int32_t dst_on_device);
/* DMVR refinement deltas of the last picture (PredictionUnit::mvdL0SubPu, 1/16 luma sample): one
 * {dx, dy} per 16x16 DMVR sub-block, PUs in descriptor order, sub-blocks in raster order inside each PU
 * (xProcessDMVR InterPrediction.cpp:2162-2296). Copies min(n, count) pairs into out and returns the
 * count (>= 0) or a negative error. Blocks until the picture's motion compensation has run. */
int vvcr_get_dmvr_deltas(vvcr_ctx *ctx, int32_t *out, int64_t n);
/* The same for a launched prepared picture (any, not only the last): waits for that picture's inter
 * stage only, so a host producer can hand a picture's refined motion to the pictures that use it as
 * collocated reference (vvcp_refine_motion) while its lane goes on with intra and the loop filters. */
int vvcr_picture_dmvr_deltas(vvcr_ctx *ctx, int32_t handle, int32_t *out, int64_t n);

/* Timing of the last vvcr_end_picture*, in ms (HIP events on the library stream): ms[0] = whole call,
 * ms[1 + k] = stage k in VVCR_STAGE_* bit order (RESID, INTER, INTRA, LMCS_INV, DBK, SAO, ALF), 0 if
 * the stage did not run. n = number of entries wanted (<= 8). */
int vvcr_last_stage_times(vvcr_ctx *ctx, float *ms, int32_t n);
/* Raw HIP stream handle (hipStream_t) of the context's first execution lane (host copies use it). */
void *vvcr_stream(vvcr_ctx *ctx);


/* ============================================================================================== *
 * Encoder RDO inner loop (BASELINE config 5): batched distortion and forward
 * transforms. They replace, for a batch of blocks at once, the per-block calls the encoder makes:
 *   vvcr_rd_*   <- RdCost::setDistParam + DistParam::distFunc (RdCost.h:181, RdCost.cpp:503 xGetSAD,
 *                  :2800 xGetHADs — the Hadamard SATD with its 2x2 .. 16x8 tiles), bit depth 10;
 *   vvcr_fwd_*  <- TrQuant::xT (TrQuant.cpp:749-824) over fastFwdTrans (TrQuant.cpp:69-74).
 * plan uploads the block list (host pointers) and returns a handle; run reads DEVICE pointers (inputs
 * resident in HBM) and is asynchronous on the context stream (vvcr_sync waits); the vvcr_rd_dist /
 * vvcr_fwd_transform forms take host pointers and block until the results are copied back.
 * ============================================================================================== */
typedef struct vvcr_rd_block {
  int64_t org_off, cur_off;        /* sample offsets of the block in the original / prediction pools */
  int32_t org_stride, cur_stride;  /* row pitch in samples */
  int32_t width, height;           /* even sizes (xGetHADs rejects odd ones) */
} vvcr_rd_block;
typedef struct vvcr_fwd_block {
  int64_t src_off;                 /* residual sample offset */
  int64_t dst_off;                 /* coefficient offset: width*height int32, row-major */
  int32_t src_stride;
  int32_t width, height;           /* 4..64 (DCT2), 4..32 (DST7 / DCT8) */
  int32_t tr_hor, tr_ver;          /* 0 DCT2, 1 DST7, 2 DCT8 */
  int32_t lfnst;                   /* non-zero: the zero-out xT applies when lfnstIdx != 0 */
} vvcr_fwd_block;
int vvcr_rd_plan(vvcr_ctx *ctx, const vvcr_rd_block *blocks, int32_t n, int32_t *plan);
int vvcr_rd_run(vvcr_ctx *ctx, int32_t plan, const int16_t *org_dev, const int16_t *cur_dev, uint32_t *sad_dev,
                uint32_t *satd_dev);
int vvcr_fwd_plan(vvcr_ctx *ctx, const vvcr_fwd_block *blocks, int32_t n, int32_t bit_depth, int32_t *plan);
int vvcr_fwd_run(vvcr_ctx *ctx, int32_t plan, const int16_t *resi_dev, int32_t *coef_dev);
int vvcr_rdo_release(vvcr_ctx *ctx, int32_t plan);
int vvcr_rd_dist(vvcr_ctx *ctx, const vvcr_rd_block *blocks, int32_t n, const int16_t *org, int64_t norg,
                 const int16_t *cur, int64_t ncur, uint32_t *sad, uint32_t *satd);
int vvcr_fwd_transform(vvcr_ctx *ctx, const vvcr_fwd_block *blocks, int32_t n, int32_t bit_depth, const int16_t *resi,
                       int64_t nresi, int32_t *coef, int64_t ncoef);

#ifdef __cplusplus
}
#endif
#endif /* VVCR_H */
