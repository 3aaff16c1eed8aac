// H.264 / AVC constant tables shared by the host bitstream library, the
// independent CPU decoder and the gfx950 HIP kernels.
//
// Every table here is transcribed from ITU-T H.264 (the clause is named on each
// table).  The reference repository (GPUs/goVideoCompressor) has no codec code
// at all: it shells out to ffmpeg at client.go:115 (`ffmpeg -i <idx>.mp4 <args>`)
// and server.go:199 (segment muxer).  This header is the first layer of the
// MI355X-native replacement for that external libx264 dependency.
//
// Usable from host C++ and HIP device code (namespace-scope constexpr arrays are
// emitted on the device when ODR-used by a kernel).
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define MIVC_HD __host__ __device__ __forceinline__
#else
#define MIVC_HD inline
#endif

namespace mivc {
namespace h264 {

// ---------------------------------------------------------------- scans
// 4x4 frame zig-zag scan (clause 8.5.6, Table 8-13): scan index -> raster
// position (x + 4*y) inside the 4x4 block.
static constexpr uint8_t kZigzag4x4[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};

// ---------------------------------------------------------------- scaling matrices (7.4.2.1.1)
// Default_4x4_Intra / _Inter (Table 7-3) and Default_8x8_Intra / _Inter (Table 7-4), in
// zig-zag scan order (index = scan position, as scaling_list() codes them)
static constexpr uint8_t kDefault4x4[2][16] = {{6, 13, 13, 20, 20, 20, 28, 28, 28, 28, 32, 32, 32, 37, 37, 42},
                                               {10, 14, 14, 20, 20, 20, 24, 24, 24, 24, 27, 27, 27, 30, 30, 34}};
static constexpr uint8_t kDefault8x8[2][64] = {
    {6,  10, 10, 13, 11, 13, 16, 16, 16, 16, 18, 18, 18, 18, 18, 23, 23, 23, 23, 23, 23, 25,
     25, 25, 25, 25, 25, 25, 27, 27, 27, 27, 27, 27, 27, 27, 29, 29, 29, 29, 29, 29, 29, 31,
     31, 31, 31, 31, 31, 33, 33, 33, 33, 33, 36, 36, 36, 36, 38, 38, 38, 40, 40, 42},
    {9,  13, 13, 15, 13, 15, 17, 17, 17, 17, 19, 19, 19, 19, 19, 21, 21, 21, 21, 21, 21, 22,
     22, 22, 22, 22, 22, 22, 24, 24, 24, 24, 24, 24, 24, 24, 25, 25, 25, 25, 25, 25, 25, 27,
     27, 27, 27, 27, 27, 28, 28, 28, 28, 28, 30, 30, 30, 30, 32, 32, 32, 33, 33, 35}};


// inverse: raster position (x + 4*y) -> scan index
static constexpr uint8_t kZigzagInv4x4[16] = {0, 1, 5, 6, 2, 4, 7, 12, 3, 8, 11, 13, 9, 10, 14, 15};

// luma4x4BlkIdx (clause 6.4.3, 8x8 Z-order) -> x,y of the 4x4 block in 4-sample units.
static constexpr uint8_t kBlkX[16] = {0, 1, 0, 1, 2, 3, 2, 3, 0, 1, 0, 1, 2, 3, 2, 3};
static constexpr uint8_t kBlkY[16] = {0, 0, 1, 1, 0, 0, 1, 1, 2, 2, 3, 3, 2, 2, 3, 3};
// inverse: raster 4x4 position (x + 4*y) -> luma4x4BlkIdx
static constexpr uint8_t kRasterToBlk[16] = {0, 1, 4, 5, 2, 3, 6, 7, 8, 9, 12, 13, 10, 11, 14, 15};

// ---------------------------------------------------------------- quantisation
// Forward quantisation multipliers MF (encoder side, not normative).  Rows: QP%6.
// Columns: position class 0 = (0,0),(0,2),(2,0),(2,2); 1 = (1,1),(1,3),(3,1),(3,3); 2 = other.
static constexpr int32_t kQuantMF[6][3] = {
    {13107, 5243, 8066}, {11916, 4660, 7490}, {10082, 4194, 6554},
    {9362, 3647, 5825},  {8192, 3355, 5243},  {7282, 2893, 4559}};
// Dequantisation normAdjust4x4 v (clause 8.5.9, eq. 8-315). Same column classes.
static constexpr int32_t kDequantV[6][3] = {
    {10, 16, 13}, {11, 18, 14}, {13, 20, 16}, {14, 23, 18}, {16, 25, 20}, {18, 29, 23}};

// position class of raster 4x4 position (x + 4*y)
static constexpr uint8_t kPosClass[16] = {0, 2, 0, 2, 2, 1, 2, 1, 0, 2, 0, 2, 2, 1, 2, 1};

// QPc as a function of qPI (clause 8.5.8, Table 8-15); qPI in [0,51].
static constexpr uint8_t kChromaQp[52] = {
    0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17,
    18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 29, 30, 31, 32, 32, 33,
    34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39};

// ---------------------------------------------------------------- deblocking
// Table 8-16: alpha'(indexA), beta'(indexB)
static constexpr uint8_t kAlpha[52] = {
    0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,   0,   0,   0,   0,   4,   4,
    5,  6,  7,  8,  9,  10, 12, 13, 15, 17, 20, 22,  25,  28,  32,  36,  40,  45,
    50, 56, 63, 71, 80, 90, 101, 113, 127, 144, 162, 182, 203, 226, 255, 255};
static constexpr uint8_t kBeta[52] = {
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  0,  0,  0,  2,  2,
    2, 3, 3, 3, 3, 4, 4, 4, 6, 6, 7,  7,  8,  8,  9,  9,  10, 10,
    11, 11, 12, 12, 13, 13, 14, 14, 15, 15, 16, 16, 17, 17, 18, 18};
// Table 8-17: tC0'(indexA, bS) for bS = 1,2,3
static constexpr uint8_t kTc0[52][3] = {
    {0, 0, 0},   {0, 0, 0},   {0, 0, 0},   {0, 0, 0},    {0, 0, 0},    {0, 0, 0},   {0, 0, 0},
    {0, 0, 0},   {0, 0, 0},   {0, 0, 0},   {0, 0, 0},    {0, 0, 0},    {0, 0, 0},   {0, 0, 0},
    {0, 0, 0},   {0, 0, 0},   {0, 0, 0},   {0, 0, 1},    {0, 0, 1},    {0, 0, 1},   {0, 0, 1},
    {0, 1, 1},   {0, 1, 1},   {1, 1, 1},   {1, 1, 1},    {1, 1, 1},    {1, 1, 1},   {1, 1, 2},
    {1, 1, 2},   {1, 1, 2},   {1, 1, 2},   {1, 2, 3},    {1, 2, 3},    {2, 2, 3},   {2, 2, 4},
    {2, 3, 4},   {2, 3, 4},   {3, 3, 5},   {3, 4, 6},    {3, 4, 6},    {4, 5, 7},   {4, 5, 8},
    {4, 6, 9},   {5, 7, 10},  {6, 8, 11},  {6, 8, 13},   {7, 10, 14},  {8, 11, 16}, {9, 12, 18},
    {10, 13, 20}, {11, 15, 23}, {13, 17, 25}};

// ---------------------------------------------------------------- CAVLC (clause 9.2)
// coeff_token, Table 9-5, indexed [table][TotalCoeff*4 + TrailingOnes].
// table 0: 0<=nC<2, 1: 2<=nC<4, 2: 4<=nC<8, 3: 8<=nC (6-bit FLC).
static constexpr uint8_t kCoeffTokenLen[4][68] = {
    {1,  0,  0,  0,  6,  2,  0,  0,  8,  6,  3,  0,  9,  8,  7,  5,  10, 9,  8,  6,  11, 10, 9,
     7,  13, 11, 10, 8,  13, 13, 11, 9,  13, 13, 13, 10, 14, 14, 13, 11, 14, 14, 14, 13, 15, 15,
     14, 14, 15, 15, 15, 14, 16, 15, 15, 15, 16, 16, 16, 15, 16, 16, 16, 16, 16, 16, 16, 16},
    {2,  0,  0,  0,  6,  2,  0,  0,  6,  5,  3,  0,  7,  6,  6,  4,  8,  6,  6,  4,  8,  7,  7,
     5,  9,  8,  8,  6,  11, 9,  9,  6,  11, 11, 11, 7,  12, 11, 11, 9,  12, 12, 12, 11, 12, 12,
     12, 11, 13, 13, 13, 12, 13, 13, 13, 13, 13, 14, 13, 13, 14, 14, 14, 13, 14, 14, 14, 14},
    {4, 0, 0, 0, 6, 4, 0, 0, 6, 5, 4, 0, 6, 5, 5, 4, 7, 5, 5,  4,  7,  5,  5,  4,  7,  6, 6, 4, 7,
     6, 6, 4, 8, 7, 7, 5, 8, 8, 7, 6, 9, 8, 8, 7, 9, 9, 8, 8,  9,  9,  9,  8,  10, 9,  9, 9, 10,
     10, 10, 10, 10, 10, 10, 10, 10, 10, 10, 10},
    {6, 0, 0, 0, 6, 6, 0, 0, 6, 6, 6, 0, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6,
     6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6}};
static constexpr uint8_t kCoeffTokenBits[4][68] = {
    {1, 0, 0, 0, 5, 1, 0, 0, 7, 4, 1, 0, 7, 6, 5, 3, 7, 6,  5,  3, 7,  6,  5, 4, 15, 6,  5, 4, 11, 14, 5, 4, 8,  10,
     13, 4, 15, 14, 9, 4, 11, 10, 13, 12, 15, 14, 9, 12, 11, 10, 13, 8, 15, 1, 9, 12, 11, 14, 13, 8, 7, 10, 9, 12, 4, 6, 5, 8},
    {3,  0, 0,  0, 11, 2,  0,  0, 7,  7,  3,  0, 7,  10, 9,  5,  7,  6, 5, 4, 4,  6, 5, 6, 7, 6, 5, 8, 15, 6, 5, 4, 11, 14,
     13, 4, 15, 10, 9, 4, 11, 14, 13, 12, 8, 10, 9, 8, 15, 14, 13, 12, 11, 10, 9, 12, 7, 11, 6, 8, 9, 8, 10, 1, 7, 6, 5, 4},
    {15, 0,  0,  0, 15, 14, 0,  0,  11, 15, 13, 0, 8, 12, 14, 12, 15, 10, 11, 11, 11, 8,  9, 10, 9, 14, 13, 9, 8, 10, 9, 8,
     15, 14, 13, 13, 11, 14, 10, 12, 15, 10, 13, 12, 11, 14, 9, 12, 8, 10, 13, 8, 13, 7, 9, 12, 9, 12, 11, 10, 5, 8, 7, 6, 1, 4, 3, 2},
    {3,  0,  0,  0,  0,  1,  0,  0,  4,  5,  6,  0,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17, 18,
     19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 38, 39, 40, 41,
     42, 43, 44, 45, 46, 47, 48, 49, 50, 51, 52, 53, 54, 55, 56, 57, 58, 59, 60, 61, 62, 63}};
// coeff_token for ChromaDCLevel with ChromaArrayType == 1 (nC == -1), [TotalCoeff*4 + T1]
static constexpr uint8_t kChromaDcCoeffTokenLen[20] = {2, 0, 0, 0, 6, 1, 0, 0, 6, 6, 3, 0, 6, 7, 7, 6, 6, 8, 8, 7};
static constexpr uint8_t kChromaDcCoeffTokenBits[20] = {1, 0, 0, 0, 7, 1, 0, 0, 4, 6, 1, 0, 3, 3, 2, 5, 2, 3, 2, 0};

// total_zeros for 4x4 blocks, Tables 9-7 / 9-8: [TotalCoeff-1][total_zeros]
static constexpr uint8_t kTotalZerosLen[15][16] = {
    {1, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 9}, {3, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 6, 6, 6, 6, 0},
    {4, 3, 3, 3, 4, 4, 3, 3, 4, 5, 5, 6, 5, 6, 0, 0}, {5, 3, 4, 4, 3, 3, 3, 4, 3, 4, 5, 5, 5, 0, 0, 0},
    {4, 4, 4, 3, 3, 3, 3, 3, 4, 5, 4, 5, 0, 0, 0, 0}, {6, 5, 3, 3, 3, 3, 3, 3, 4, 3, 6, 0, 0, 0, 0, 0},
    {6, 5, 3, 3, 3, 2, 3, 4, 3, 6, 0, 0, 0, 0, 0, 0}, {6, 4, 5, 3, 2, 2, 3, 3, 6, 0, 0, 0, 0, 0, 0, 0},
    {6, 6, 4, 2, 2, 3, 2, 5, 0, 0, 0, 0, 0, 0, 0, 0}, {5, 5, 3, 2, 2, 2, 4, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {4, 4, 3, 3, 1, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, {4, 4, 2, 1, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {3, 3, 1, 2, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, {2, 2, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}};
static constexpr uint8_t kTotalZerosBits[15][16] = {
    {1, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 1}, {7, 6, 5, 4, 3, 5, 4, 3, 2, 3, 2, 3, 2, 1, 0, 0},
    {5, 7, 6, 5, 4, 3, 4, 3, 2, 3, 2, 1, 1, 0, 0, 0}, {3, 7, 5, 4, 6, 5, 4, 3, 3, 2, 2, 1, 0, 0, 0, 0},
    {5, 4, 3, 7, 6, 5, 4, 3, 2, 1, 1, 0, 0, 0, 0, 0}, {1, 1, 7, 6, 5, 4, 3, 2, 1, 1, 0, 0, 0, 0, 0, 0},
    {1, 1, 5, 4, 3, 3, 2, 1, 1, 0, 0, 0, 0, 0, 0, 0}, {1, 1, 1, 3, 3, 2, 2, 1, 0, 0, 0, 0, 0, 0, 0, 0},
    {1, 0, 1, 3, 2, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0}, {1, 0, 1, 3, 2, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {0, 1, 1, 2, 1, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, {0, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {0, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, {0, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}};
// total_zeros for 2x2 chroma DC (Table 9-9a): [TotalCoeff-1][total_zeros]
static constexpr uint8_t kChromaDcTotalZerosLen[3][4] = {{1, 2, 3, 3}, {1, 2, 2, 0}, {1, 1, 0, 0}};
static constexpr uint8_t kChromaDcTotalZerosBits[3][4] = {{1, 1, 1, 0}, {1, 1, 0, 0}, {1, 0, 0, 0}};
// run_before, Table 9-10: [min(zerosLeft,7)-1][run_before]
static constexpr uint8_t kRunBeforeLen[7][15] = {
    {1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, {1, 2, 2, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {2, 2, 2, 2, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, {2, 2, 2, 3, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {2, 2, 3, 3, 3, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0}, {2, 3, 3, 3, 3, 3, 3, 0, 0, 0, 0, 0, 0, 0, 0},
    {3, 3, 3, 3, 3, 3, 3, 4, 5, 6, 7, 8, 9, 10, 11}};
static constexpr uint8_t kRunBeforeBits[7][15] = {
    {1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, {1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {3, 2, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, {3, 2, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {3, 2, 3, 2, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, {3, 0, 1, 3, 2, 5, 4, 0, 0, 0, 0, 0, 0, 0, 0},
    {7, 6, 5, 4, 3, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1}};

// coded_block_pattern mapping (Table 9-4, ChromaArrayType 1/2): codeNum -> cbp
static constexpr uint8_t kGolombToIntraCbp[48] = {
    47, 31, 15, 0,  23, 27, 29, 30, 7,  11, 13, 14, 39, 43, 45, 46,
    16, 3,  5,  10, 12, 19, 21, 26, 28, 35, 37, 42, 44, 1,  2,  4,
    8,  17, 18, 20, 24, 6,  9,  22, 25, 32, 33, 34, 36, 40, 38, 41};
static constexpr uint8_t kGolombToInterCbp[48] = {
    0,  16, 1,  2,  4,  8,  32, 3,  5,  10, 12, 15, 47, 7,  11, 13,
    14, 6,  9,  31, 35, 37, 42, 44, 33, 34, 36, 40, 39, 43, 45, 46,
    17, 18, 20, 24, 19, 21, 26, 28, 23, 27, 29, 30, 22, 25, 38, 41};

// inverse of the above: cbp -> codeNum
static constexpr uint8_t kIntraCbpToCode[48] = {3, 29, 30, 17, 31, 18, 37, 8, 32, 38, 19, 9, 20, 10, 11, 2, 16, 33, 34, 21, 35, 22, 39, 4, 36, 40, 23, 5, 24, 6, 7, 1, 41, 42, 43, 25, 44, 26, 46, 12, 45, 47, 27, 13, 28, 14, 15, 0};
static constexpr uint8_t kInterCbpToCode[48] = {0, 2, 3, 7, 4, 8, 17, 13, 5, 18, 9, 14, 10, 15, 16, 11, 1, 32, 33, 36, 34, 37, 44, 40, 35, 45, 38, 41, 39, 42, 43, 19, 6, 24, 25, 20, 26, 21, 46, 28, 27, 47, 22, 29, 23, 30, 31, 12};

// ---------------------------------------------------------------- helpers
MIVC_HD int clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }
MIVC_HD int clip1(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }
MIVC_HD int chroma_qp(int qpy, int offset) { return kChromaQp[clip3(0, 51, qpy + offset)]; }

// 6-tap half-sample filter tap sum (clause 8.4.2.2.1): E - 5F + 20G + 20H - 5I + J
MIVC_HD int tap6(int e, int f, int g, int h, int i, int j) { return e - 5 * f + 20 * g + 20 * h - 5 * i + j; }

// Inverse 4x4 core transform of the decoder (clause 8.5.12.2): rows first, then
// columns, then (x + 32) >> 6.  d is raster (x + 4*y), modified in place to the
// residual r.
MIVC_HD void inverse_core4x4(int* d) {
  for (int y = 0; y < 4; ++y) {
    int* r = d + 4 * y;
    int e0 = r[0] + r[2], e1 = r[0] - r[2];
    int e2 = (r[1] >> 1) - r[3], e3 = r[1] + (r[3] >> 1);
    r[0] = e0 + e3; r[1] = e1 + e2; r[2] = e1 - e2; r[3] = e0 - e3;
  }
  for (int x = 0; x < 4; ++x) {
    int c0 = d[x], c1 = d[x + 4], c2 = d[x + 8], c3 = d[x + 12];
    int g0 = c0 + c2, g1 = c0 - c2;
    int g2 = (c1 >> 1) - c3, g3 = c1 + (c3 >> 1);
    d[x] = (g0 + g3 + 32) >> 6;
    d[x + 4] = (g1 + g2 + 32) >> 6;
    d[x + 8] = (g1 - g2 + 32) >> 6;
    d[x + 12] = (g0 - g3 + 32) >> 6;
  }
}

// Scaling of a 4x4 residual (non-DC path, flat weights; clause 8.5.12.1):
// d = c * v << (qp/6).  Valid for every qP in [0,51] with flat scaling lists.
MIVC_HD int dequant_coef(int c, int qp, int raster_pos) {
  return (c * kDequantV[qp % 6][kPosClass[raster_pos]]) << (qp / 6);
}

}  // namespace h264
}  // namespace mivc
