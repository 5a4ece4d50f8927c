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
/* info[0..9] = poc, slice type of the first slice (0 B, 1 P, 2 I), width, height, ctu_log2, bit depth,
 * number of slices, temporal id, NAL unit type, slice QP. Returns the number of fields (10). */
int vvcp_picture_info(const vvcp_stream *s, int32_t idx, int32_t *info, int32_t n);
int vvcp_parse_picture(vvcp_stream *s, int32_t idx);

/* Parsed rows of a picture (after vvcp_parse_picture): copies min(cap, count) entries to dst (dst may be
 * NULL) and returns count. Motion vectors of vvcr_pu are not derived by the parse pass. */
#define VVCP_ROWS_CU 0        /* vvcr_cu */
#define VVCP_ROWS_PU 1        /* vvcr_pu */
#define VVCP_ROWS_TU 2        /* vvcr_tu */
#define VVCP_ROWS_COEF 3      /* int32 coefficient levels */
#define VVCP_ROWS_SAO 4       /* vvcr_sao [n_ctb][3], merges resolved */
#define VVCP_ROWS_ALF_EN0 5   /* uint8 [n_ctb], components 0..2 at 5..7 */
#define VVCP_ROWS_ALF_ALT0 8  /* uint8 [n_ctb], components 0..2 at 8..10 */
#define VVCP_ROWS_ALF_FSET 11 /* int16 [n_ctb] luma filter set */
#define VVCP_ROWS_CCALF0 12   /* uint8 [n_ctb], Cb at 12, Cr at 13 */
int64_t vvcp_picture_rows(const vvcp_stream *s, int32_t idx, int32_t what, void *dst, int64_t cap);

#ifdef __cplusplus
}
#endif
#endif /* VVCP_H */
