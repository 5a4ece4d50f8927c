/*
 * vvcp.h — C-ABI of libvvcr's host bitstream parser: the producer of the vvcr_cu / vvcr_pu / vvcr_tu
 * descriptor rows of include/vvcr.h straight from a VVC (VTM-7.3 draft) Annex-B bitstream.
 *
 * It replaces the reference decoder's parsing front end for the drop-in path:
 *   DecApp::decode -> DecLib::decode (DecoderLib/DecLib.cpp) NAL and header handling  ->  vvcp_open
 *   DecSlice::decompressSlice -> CABACReader::coding_tree_unit (CABACReader.cpp:136)   ->  vvcp_parse_picture
 * vvcp_open reads every NAL unit and header (parameter sets, APS, picture and slice headers, reference
 * lists) serially; vvcp_parse_picture runs the CABAC pass of one picture, which depends on no other
 * picture, so different pictures may be parsed on different threads at once.
 * Same conventions as vvcr.h: 0 / count on success, negative VVCR_E_* codes on failure,
 * vvcp_last_error() (per thread) gives the message.
 */
#ifndef VVCP_H
#define VVCP_H

#include <stddef.h>
#include <stdint.h>

#include "vvcr.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct vvcp_stream vvcp_stream;

int vvcp_open(const uint8_t *data, size_t n, vvcp_stream **out);
int vvcp_close(vvcp_stream *s);
const char *vvcp_last_error(void);
int vvcp_num_pictures(const vvcp_stream *s);
/* info[0..15] = poc, slice type of the first slice (0 B, 1 P, 2 I), width, height, ctu_log2, bit depth,
 * number of slices, temporal id, NAL unit type, slice QP, conformance window left / right / top / bottom
 * offsets in luma samples, pic_output_flag, non-reference picture flag. Returns the number of fields (16). */
int vvcp_picture_info(const vvcp_stream *s, int32_t idx, int32_t *info, int32_t n);
int vvcp_parse_picture(vvcp_stream *s, int32_t idx);
/* The decoded picture hash SEI that follows picture idx (SEIReader::xParseSEIDecodedPictureHash,
 * SEIread.cpp:420): returns its hash_type (0 MD5, 1 CRC, 2 checksum) and copies the per-component
 * hashes (16 / 2 / 4 bytes each, Y Cb Cr) to out[0..n); -1 when the picture has none. */
int vvcp_picture_hash(const vvcp_stream *s, int32_t idx, uint8_t *out, int32_t n);
/* Per-rank parsing of a spatially sharded decode (BASELINE config 4): the CABAC pass of every later
 * vvcp_parse_picture covers only the tiles holding luma rows [y0, y1), each up to the CTU row holding
 * y1 - 1 (a tile's substreams are decoded from its start, DecSlice.cpp:106-114, so a tile above is parsed
 * whole; one below only as deep as needed). Motion derivation and planning then see the CUs of those rows
 * (the shard, its deblocking halo and the tiles' HMVP / TMVP neighbourhood, all inside the tiles); the
 * DMVR delta list of such a picture is the sub-list of its parsed PUs (vvcp_dmvr_split). y1 <= y0: every
 * row (the default). */
int vvcp_set_parse_rows(vvcp_stream *s, int32_t y0, int32_t y1);
/* The delta rows (vvcp_refine_motion layout) of a derived picture's DMVR PUs above luma row y0, in
 * [y0, y1) and from y1 on, among the PUs its CABAC pass covered: out[0..2]. With tile-row shards a
 * rank's list is then its upper neighbour's last out[0] rows, its own rows and its lower neighbour's
 * first out[2] rows. */
int vvcp_dmvr_split(const vvcp_stream *s, int32_t idx, int32_t y0, int32_t y1, int64_t *out);

/* Motion derivation of a parsed picture (DecCu::xDeriveCUMV, DecCu.cpp:878, with the merge / AMVP /
 * affine / SbTMVP / GEO / MMVD candidate tools of UnitTools.cpp and the history table): fills the MV
 * fields of its vvcr_cu / vvcr_pu rows, the 4x4 motion field and the GEO rows. Pictures must be derived
 * in decoding order, and every earlier picture must have been refined (vvcp_refine_motion) first, since
 * it may be the collocated reference. */
int vvcp_derive_motion(vvcp_stream *s, int32_t idx);
/* CS::setRefinedMotionField (UnitTools.cpp:68): records the motion of a derived picture as later
 * pictures' temporal candidates see it, with the DMVR deltas of its PUs (vvcr_get_dmvr_deltas layout:
 * n (dx, dy) pairs, PUs with pu.dmvr in row order, 16x16 sub-blocks in raster order). deltas may be
 * NULL when no PU of the picture refines. */
int vvcp_refine_motion(vvcp_stream *s, int32_t idx, const int32_t *deltas, int64_t n);

/* Picture parameters of the reconstruction path (include/vvcr.h vvcr_pic_params) from the parsed
 * headers: everything except pp->slot and pp->ref_slot, which the caller's DPB assigns. Slice-level
 * fields are the last slice's; slices of one picture must share their reference lists. */
int vvcp_picture_params(const vvcp_stream *s, int32_t idx, vvcr_pic_params *pp);
/* ALF / CC-ALF filters of a picture as vvcr_alf takes them (AdaptiveLoopFilter::reconstructCoeffAPSs,
 * AdaptiveLoopFilter.cpp:620): luma_coef / luma_clip [sets][25][13] for the 16 fixed sets then the
 * slice's luma APS sets (at most max_sets copied), chroma [8][7], cc_coef [2][4][8]. Any pointer may be
 * NULL. Returns the number of luma sets (16 + luma APS count). */
int vvcp_alf_filters(const vvcp_stream *s, int32_t idx, int16_t *luma_coef, int16_t *luma_clip, int32_t max_sets,
                     int16_t *chroma_coef, int16_t *chroma_clip, int16_t *cc_coef);

/* Plans a parsed and motion-derived picture for the reconstruction path: vvcr_picture_create with
 * vvcp_picture_params plus the caller's DPB slots (slot; ref_slot[l * VVCR_MAX_REF + r] for the active
 * references), vvcr_picture_submit of the rows, vvcr_picture_set_loop_filter_params (SAO, ALF / CC-ALF)
 * and vvcr_picture_plan(stage_mask), in native code. On success *out is the planned picture (the
 * caller uploads it with vvcr_prepare_planned and frees it with vvcr_picture_destroy). Thread-safe for
 * different pictures. The picture's TU rows, coefficient pool and motion rows are handed over, not
 * copied: afterwards vvcp_picture_rows returns them empty and the picture cannot be planned again. */
int vvcp_plan_picture(vvcp_stream *s, int32_t idx, const vvcr_seq_params *sp, int32_t slot, const int32_t *ref_slot,
                      uint32_t stage_mask, vvcr_picture **out);
/* vvcp_plan_picture for the spatial shard of luma rows [shard_y0, shard_y1) (vvcr_pic_params::shard_y0 /
 * shard_y1; 0, 0 = the whole picture). */
int vvcp_plan_picture_rows(vvcp_stream *s, int32_t idx, const vvcr_seq_params *sp, int32_t slot, const int32_t *ref_slot,
                           uint32_t stage_mask, int32_t shard_y0, int32_t shard_y1, vvcr_picture **out);

/* The whole decode loop in native code (DecApp::decode, App/DecoderApp/DecApp.cpp:76-200, with this
 * parser and libvvcr in place of DecLib): CABAC of every picture on `threads` parser threads, then per
 * picture in decoding order the refined motion of its pending references (their DMVR deltas from the
 * GPU), motion derivation, vvcp_plan_picture, vvcr_prepare_planned and vvcr_launch_picture on ctx.
 * DPB slots [slot_base, slot_base + num_slots) of ctx (created with ctx_slots slots) hold the pictures;
 * a picture keeps its slot until its last use as a reference and its output. on_output(user, idx, poc,
 * slot) is called in output order (POC order within each coded video sequence) as soon as the picture
 * may be output, its samples still in the slot (vvcr_write_output / vvcr_read_picture wait for them).
 * handles_out (optional, [number of pictures]): the prepared pictures are kept and their handles
 * written there in decoding order (the caller may launch them again and must release them).
 * phase_seconds (optional, [VVCP_DECODE_PHASES]) accumulates the time spent per phase. Several
 * decodes may run on several threads at once against one context, on disjoint slot ranges.
 * Returns 0 or a negative VVCR_E_* code (vvcp_last_error() of the calling thread). */
typedef void (*vvcp_output_fn)(void *user, int32_t idx, int32_t poc, int32_t slot);
enum {
  VVCP_PHASE_PARSE = 0,       /* CABAC on the parser threads (summed) */
  VVCP_PHASE_PARSE_WAIT,      /* decode loop waiting for the parser threads */
  VVCP_PHASE_DMVR_WAIT,       /* waiting for reference pictures' DMVR deltas, refining their motion */
  VVCP_PHASE_DERIVE,          /* motion derivation */
  VVCP_PHASE_PLAN,            /* picture parameters, ALF filters, work lists, intra plan, deblocking edges */
  VVCP_PHASE_PREPARE,         /* upload (vvcr_prepare_planned) */
  VVCP_PHASE_LAUNCH,          /* vvcr_launch_picture */
  VVCP_PHASE_OUTPUT,          /* on_output callbacks */
  VVCP_DECODE_PHASES
};
typedef struct vvcp_decode_params {
  int32_t slot_base, num_slots, ctx_slots;
  int32_t threads;
  uint32_t stage_mask;
  vvcp_output_fn on_output;
  void *user;
  int32_t *handles_out;
  double *phase_seconds;
} vvcp_decode_params;
int vvcp_decode(vvcp_stream *s, vvcr_ctx *ctx, const vvcp_decode_params *p);
/* The plan vvcp_decode follows: the DPB slot of every picture (slots[number of pictures]) and the
 * decode indices in output order (out_order[number of pictures]); either may be NULL. Returns the
 * number of output pictures. */
int vvcp_decode_plan(const vvcp_stream *s, int32_t slot_base, int32_t num_slots, int32_t *slots, int32_t *out_order);
/* vvcp_decode's prepared-handle release policy simulated on the stream's reference structure (decoding
 * order, every picture launched after its derivation, every picture assumed to have DMVR sub-blocks):
 * the largest number of handles alive at once when `keep` are kept beyond the policy. Host only. */
int vvcp_decode_live_bound(const vvcp_stream *s, int32_t slot_base, int32_t num_slots, int32_t keep);
/* The frame batching vvcp_decode applies (vvcr_launch_pictures; VVCP_MC_BATCH=k caps a group at k pictures,
 * 1 turns it off): first[i] = k for the first picture of a group of k launched together, 0 for a later
 * member, 1 for a picture launched alone (first may be NULL). Returns the number of groups of > 1. Host only. */
int vvcp_decode_batches(const vvcp_stream *s, int32_t slot_base, int32_t num_slots, int32_t *first);

/* Parsed rows of a picture (after vvcp_parse_picture): copies min(cap, count) entries to dst (dst may be
 * NULL) and returns count. MV fields of vvcr_cu / vvcr_pu hold parsed values until vvcp_derive_motion. */
#define VVCP_ROWS_CU 0        /* vvcr_cu */
#define VVCP_ROWS_PU 1        /* vvcr_pu */
#define VVCP_ROWS_TU 2        /* vvcr_tu */
#define VVCP_ROWS_COEF 3      /* int32 coefficient levels */
#define VVCP_ROWS_SAO 4       /* vvcr_sao [n_ctb][3], merges resolved */
#define VVCP_ROWS_ALF_EN0 5   /* uint8 [n_ctb], components 0..2 at 5..7 */
#define VVCP_ROWS_ALF_ALT0 8  /* uint8 [n_ctb], components 0..2 at 8..10 */
#define VVCP_ROWS_ALF_FSET 11 /* int16 [n_ctb] luma filter set */
#define VVCP_ROWS_CCALF0 12   /* uint8 [n_ctb], Cb at 12, Cr at 13 */
#define VVCP_ROWS_MOTION 14   /* vvcr_motion [h/4][w/4] (after vvcp_derive_motion) */
#define VVCP_ROWS_GEO 15      /* vvcr_geo (after vvcp_derive_motion) */
int64_t vvcp_picture_rows(const vvcp_stream *s, int32_t idx, int32_t what, void *dst, int64_t cap);

#ifdef __cplusplus
}
#endif
#endif /* VVCP_H */
