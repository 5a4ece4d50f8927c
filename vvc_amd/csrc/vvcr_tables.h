// vvcr_tables.h — VVC constant tables used by the HIP kernels (values are the standard's constants,
// as listed in VTM 7.3: InterpolationFilter.cpp:57-332).
#pragma once
#include <cstdint>

// 8-tap luma filters, 16 phases (InterpolationFilter.cpp:77 m_lumaFilter)
#define VVCR_LUMA_FILTER_TABLE {                                            \
  {  0, 0,   0, 64,  0,   0,  0,  0 }, {  0, 1,  -3, 63,  4,  -2,  1,  0 }, \
  { -1, 2,  -5, 62,  8,  -3,  1,  0 }, { -1, 3,  -8, 60, 13,  -4,  1,  0 }, \
  { -1, 4, -10, 58, 17,  -5,  1,  0 }, { -1, 4, -11, 52, 26,  -8,  3, -1 }, \
  { -1, 3,  -9, 47, 31, -10,  4, -1 }, { -1, 4, -11, 45, 34, -10,  4, -1 }, \
  { -1, 4, -11, 40, 40, -11,  4, -1 }, { -1, 4, -10, 34, 45, -11,  4, -1 }, \
  { -1, 4, -10, 31, 47,  -9,  3, -1 }, { -1, 3,  -8, 26, 52, -11,  4, -1 }, \
  {  0, 1,  -5, 17, 58, -10,  4, -1 }, {  0, 1,  -4, 13, 60,  -8,  3, -1 }, \
  {  0, 1,  -3,  8, 62,  -5,  2, -1 }, {  0, 1,  -2,  4, 63,  -3,  1,  0 } }

// 6-tap (in 8) luma filters for 4x4 affine sub-blocks (InterpolationFilter.cpp:57 m_lumaFilter4x4)
#define VVCR_LUMA4x4_FILTER_TABLE {                                         \
  {  0, 0,   0, 64,  0,   0,  0,  0 }, {  0, 1,  -3, 63,  4,  -2,  1,  0 }, \
  {  0, 1,  -5, 62,  8,  -3,  1,  0 }, {  0, 2,  -8, 60, 13,  -4,  1,  0 }, \
  {  0, 3, -10, 58, 17,  -5,  1,  0 }, {  0, 3, -11, 52, 26,  -8,  2,  0 }, \
  {  0, 2,  -9, 47, 31, -10,  3,  0 }, {  0, 3, -11, 45, 34, -10,  3,  0 }, \
  {  0, 3, -11, 40, 40, -11,  3,  0 }, {  0, 3, -10, 34, 45, -11,  3,  0 }, \
  {  0, 3, -10, 31, 47,  -9,  2,  0 }, {  0, 2,  -8, 26, 52, -11,  3,  0 }, \
  {  0, 1,  -5, 17, 58, -10,  3,  0 }, {  0, 1,  -4, 13, 60,  -8,  2,  0 }, \
  {  0, 1,  -3,  8, 62,  -5,  1,  0 }, {  0, 1,  -2,  4, 63,  -3,  1,  0 } }

// alternative half-pel luma filter (InterpolationFilter.cpp:183 m_lumaAltHpelIFilter)
#define VVCR_LUMA_ALT_HPEL { 0, 3, 9, 20, 20, 9, 3, 0 }

// 4-tap chroma filters, 32 phases (InterpolationFilter.cpp:184 m_chromaFilter)
#define VVCR_CHROMA_FILTER_TABLE {                                                            \
  {  0, 64,  0,  0 }, { -1, 63,  2,  0 }, { -2, 62,  4,  0 }, { -2, 60,  7, -1 },             \
  { -2, 58, 10, -2 }, { -3, 57, 12, -2 }, { -4, 56, 14, -2 }, { -4, 55, 15, -2 },             \
  { -4, 54, 16, -2 }, { -5, 53, 18, -2 }, { -6, 52, 20, -2 }, { -6, 49, 24, -3 },             \
  { -6, 46, 28, -4 }, { -5, 44, 29, -4 }, { -4, 42, 30, -4 }, { -4, 39, 33, -4 },             \
  { -4, 36, 36, -4 }, { -4, 33, 39, -4 }, { -4, 30, 42, -4 }, { -4, 29, 44, -5 },             \
  { -4, 28, 46, -6 }, { -3, 24, 49, -6 }, { -2, 20, 52, -6 }, { -2, 18, 53, -5 },             \
  { -2, 16, 54, -4 }, { -2, 15, 55, -4 }, { -2, 14, 56, -4 }, { -2, 12, 57, -3 },             \
  { -2, 10, 58, -2 }, { -1,  7, 60, -2 }, {  0,  4, 62, -2 }, {  0,  2, 63, -1 } }

// bilinear filter in 1/16 precision for DMVR search (InterpolationFilter.cpp:314 m_bilinearFilterPrec4)
#define VVCR_BILINEAR_PREC4_TABLE {                                                            \
  { 16, 0 }, { 15, 1 }, { 14, 2 }, { 13, 3 }, { 12, 4 }, { 11, 5 }, { 10, 6 }, { 9, 7 },       \
  { 8, 8 }, { 7, 9 }, { 6, 10 }, { 5, 11 }, { 4, 12 }, { 3, 13 }, { 2, 14 }, { 1, 15 } }

// BCW weights for list 1 (Rom.cpp:190 g_BcwWeights); list 0 weight = 8 - w1
#define VVCR_BCW_W1 { -2, 3, 4, 5, 10 }
