// orbx_internal.h — host/device shared layout of the MI355X ORB front-end.
//
// HBM layout (one extractor handle, batch of B same-sized images):
//   pyr   [B][Σ_l pitch_l*h_l] u8    image pyramid (mvImagePyramid), level 0 = input copy
//   blur  [B][Σ_l pitch_l*h_l] u8    7x7 Gaussian of every level (descriptor sampling)
//   ccnt  [B][n_cells]         i32   FAST candidates per cell
//   cand  [B][Σ cells cap_c]   u32   packed candidates (x:12 | y:12 | score:8), raster order
//   ocnt  [B][L]               i32   keypoints per level after the octree
//   okp   [B][Σ_l out_cap_l]   u32   packed octree survivors in list order
//   operm [B][Σ_l out_cap_l]   u16   k_orient_desc's processing order (list indices), after okp
//   kps   [B][kp_cap]          orbx_keypoint (cv::KeyPoint layout), level-major
//   desc  [B][kp_cap][32]      u8
//   nkp   [B]                  i32
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#define ORBX_MAX_LEVELS 16
#define ORBX_EDGE 19
#define ORBX_MIN_BORDER 16   // EDGE_THRESHOLD - 3, src/ORBextractor.cc:785
#define ORBX_MAX_DEVICES 64  // per-device kernel attribute caches (prepare_kernels, kfdb)

namespace orbx {

struct LevelGeom {
    int w, h, pitch;
    long long off;          // byte offset of the level inside one image's pyramid block
    float scale, inv_scale;
    int nfeat;              // mnFeaturesPerLevel
    int ncols, nrows, wcell, hcell;
    int cell_begin, ncells; // range in the cell table
    long long cand_off;     // u32 offset of the level's first cell slot in one image's block
    int cand_cap;           // Σ cell caps of the level
    int n_ini;              // DistributeOctTree root count (0: level yields nothing)
    float hx;               // root width (float, as the reference)
    int out_off, out_cap;   // octree output slots
    int kp_level_cap;       // == out_cap
    int rtab_off;           // resize tables (level>0): offset into the i16 table buffer
    int xmax;               // resize: first dx whose right tap is out of range
    int rsimd_end;          // resize: SSE2 vertical loop end (0 in scalar mode)
    int bsimd_end;          // blur: SSE2 column loop end (0 in scalar mode)
    int area2;              // resize at exactly 1/2: INTER_AREA 2x2 fast path
    int copy;               // resize to the same size: plain copy
    int patch_size;         // (int)(31*scale)
    int ntx, nty;           // k_level tiles of this level
    int ctab, rowtab;       // k_level: byte offsets of the level's column / row tables
    int stereo_win;         // k_stereo: row half-window of the octave-l buckets (ceil(2 scale) + 2)
    // k_level_strip (orbx_pyramid.hip): column strips walked row by row
    int strip;              // 1: this level runs k_level_strip, 0: the tiled k_level
    int snh;                // half-wave strips across (SW_PX output pixels each)
    int snw;                // waves across (ceil(snh / 2)); the strip height (rows per strip)
                            // is a launch argument chosen per call from its batch size
    int stab, srow;         // byte offsets of the strip lane table / row table in ltab
};

// k_level tiling (orbx_pyramid.hip): 128 x 32 output tile, staged with a 4-byte / 3-row halo.
#define OD_NK 8               // keypoints per wave in k_orient_desc (<= 64)
// k_octree: one launch over all levels under one LDS budget per workgroup, the
// blocks in level-major order so the long level-0 lists start first and the shorter lists of
// levels 1.. fill the CUs behind them; a level whose candidates exceed the budget's kcap keeps
// them in global scratch.  B = 512, two runs each (profiles/r03_ab_octree_merged.txt): merged
// level-major at 40 KB 0.322-0.323 ms, two launches (level 0, then levels 1..) at 40 KB
// 0.335-0.339, merged in (image, level) order 0.536-0.542, merged level-major at 52 KB 0.358-0.361
#define OCT_LDS_KB 40       // four workgroups per CU
// Default side branch of an extraction (orbx_extractor_set_overlap): the first FAST_SIDE_LV
// levels' FAST (FAST_SIDE 1), + octree (2), + orientation / descriptors (3) on the handle's
// second stream, forked before level FAST_SIDE_AT's launch; 0 = every kernel on one stream.
// B = 512 (profiles/r03_ab_side_*.txt): one stream 4.66-4.68 ms per step; mode 3 forked at
// level 3, 4.47 ms
#define FAST_SIDE 3
#define FAST_SIDE_AT 3
#define FAST_SIDE_LV 1
// Layout of the blurred pyramid (read only by k_orient_desc's rBRIEF patches and the
// orbx_blur_level readback): 16x4-pixel tiles of 64 bytes (one sector), row-major inside the
// tile, tiles row-major over the level (pitch / 16 tiles per band of 4 rows: the level keeps
// the raw pyramid's pitch, a multiple of 64, and its offset; levels are allocated in whole
// bands).  A 37x37 rBRIEF patch touches 30-40 sectors instead of ~55 row-major.
__host__ __device__ inline uint32_t blur_off(int x, int y, int pitch, int h) {
    (void)h;
    return (uint32_t)(y >> 2) * (uint32_t)(4 * pitch) + ((uint32_t)(x >> 4) << 6) +
           ((uint32_t)(y & 3) << 4) + (uint32_t)(x & 15);
}
#define LT_W 128              // output tile width  (32 groups of 4)
#define LT_H 32               // output tile height
#define LT_G 34               // halo groups per row: x = X0-4 .. X0+131
#define LT_HR (LT_H + 6)      // halo rows: y = Y0-3 .. Y0+LT_H+2

// Per-tile-column tables of k_level (host-built, build_geometry): the staged source window's
// x range and, per halo group of 4 pixels, the source columns, flags and resize alphas.
struct LevelColTab {
    int32_t x0, ww, pad0, pad1;
    uint32_t cgrp[2 * LT_G];  // 4 x u16 source column (window relative)
    uint32_t cinf[LT_G];      // 2 bits/pixel (xmax, rsimd) | 0x100 contig | 0x200 simple
                              // | 0x1000 << j: pixel j's taps sit in dwords 1-2
    uint32_t pad2[2];
    uint32_t calp[4 * LT_G];  // 4 x (alpha0 | alpha1 << 16); (2048, 0) right of xmax
    uint32_t csel[4 * LT_G];  // 4 x v_perm selector of the pixel's 2 taps (see k_level)
};
// Per-tile-row tables: the window's y range and, per halo row, source rows and betas.
struct LevelRowTab {
    int32_t y0, wh, pad0, pad1;
    uint32_t rinf[2 * LT_HR]; // (ry0 | ry1 << 16, beta0 | beta1 << 16)
};

// k_pyr_chain: one workgroup per (tile, image) computes its tile of every level.  Per level:
// the owned output rectangle [ox0, ox1) x [oy0, oy1) (level pixels and blurred pixels it
// stores; the owned rectangles of a level partition it, ox0 a multiple of 4) and the
// footprint [fx0, fx1] x [fy0, fy1] it computes into LDS: the owned rectangle + the blur's
// 3-pixel halo, and every source pixel the next level's footprint reads (fx0 a multiple of
// 4).  An empty footprint has fx1 < fx0.
struct ChainRect {
    int16_t ox0, ox1, oy0, oy1, fx0, fx1, fy0, fy1;
};
// LDS row of a footprint: 4 bytes of left pad (x = fx0 - 4 .. fx0 - 1: the reflected columns
// left of the image), the footprint, and 8 bytes of slack (the reflected columns right of it,
// the resize's third dword)
__host__ __device__ inline int chain_pitch(int fw) { return ((fw + 3) & ~3) + 12; }
// LDS words of a level's k_pyr_chain tables (ng column groups, fh rows): per group a base word,
// padded to a multiple of 4, then 4 v_perm selectors and 4 alpha pairs; per row two words
// (fh rounded up to even, so every level's tables start 16-byte aligned)
__host__ __device__ inline int chain_level_words(int ng, int fh) {
    return ((ng + 3) & ~3) + 8 * ng + 2 * ((fh + 1) & ~1);
}
#define CHAIN_TW 80    // k_pyr_chain: level-0 tile width / height targets (tiles per image =
#define CHAIN_TH 48    // ceil(w / CHAIN_TW) x ceil(h / CHAIN_TH))

// k_level_strip: a wave walks two half-strips (lanes 0-31, 32-63) down the level, one row per
// step.  Lane q of a half-strip at X0 holds the 4-pixel group x = X0 - 4 + 4q; lanes 1..SW_OUT
// write output.  Per lane (host-built, reflection and clamping folded in):
//   mode 0 (level 0): base = the group's smallest reflected input column, sel = 4 byte
//     offsets from base;
//   mode 3 (INTER_LINEAR): base = smallest source tap column, psel = per-pixel v_perm selectors
//     of the two taps relative to base, alp = 16 x alphas ((2048, 0) right of xmax), flags =
//     2 bits per pixel (right tap in range, SSE2 vertical form).
// Row table per level: rows y = -3 .. h + 2, 4 dwords each: mode 3 the byte offsets of the
// two source rows in level l-1 and (beta0 | beta1 << 16); mode 0 the reflected input row.
#define STRIP_TH 64   // output rows per strip (<= 122: the row table sits in two registers)
#define SW_OUT 30
#define SW_PX (4 * SW_OUT)
struct StripLane {
    uint32_t base, flags, sel, pad;
    uint32_t alp[4];
    uint32_t psel[4];
};

// 32 bytes, 16-byte aligned: a wave-uniform cells[i] is two scalar dwordx4 loads (a 20-byte
// record had one field fetched by a vector load, whose vmcnt(0) wait also drained the wave's
// in-flight ROI prefetch and stores)
struct alignas(16) CellDesc {
    int16_t level, ini_x, ini_y, cols, rows, pad;
    int32_t slot;           // u32 offset of this cell's candidate slot (per image block)
    int32_t cap;            // slot capacity
    int32_t pad2[3];
};
static_assert(sizeof(CellDesc) == 32, "CellDesc layout");

struct Geometry {
    int width, height, nlevels;
    int n_cells;            // cells over all levels
    int kp_cap;             // Σ_l out_cap
    long long pyr_bytes;    // per image
    long long cand_words;   // per image
    int out_words;          // per image (Σ out_cap)
    int max_ncand_level;    // max cand_cap over levels
    int max_out_cap;
    int max_roi_bytes;      // largest FAST cell ROI (rows*cols)
    int max_mbuf_bytes;     // largest FAST score buffer ((dh+2)*(dw+2)), dword padded
    int max_cell_px;        // largest FAST detection region (dh*dw)
    int blur_tiles;         // Σ_l ceil(w/64)*ceil(h/16)
    int orient_blocks;      // Σ_l ceil(out_cap / (4 * OD_NK))
    int blur_tile_begin[ORBX_MAX_LEVELS + 1];
    int orient_block_begin[ORBX_MAX_LEVELS + 1];
    int taps[7];            // cvRound(getGaussianKernel(7, 2, CV_32F) * 256)
    int umax[16];           // src/ORBextractor.cc:454-469
    int ini_th, min_th;     // FAST thresholds, clamped to [0, 255]
    int stereo_ob;          // k_stereo bucket groups: nlevels (octave, row), or 1 (row) if LDS is short
    int ltw, lth;           // k_level output tile
    int win_cap;            // k_level: largest staged source window (bytes)
    // k_pyr_chain (small batches: every level in one launch, see orbx_pyramid.hip)
    int chain_ok;           // 1: every level l >= 1 is INTER_LINEAR and the LDS fits
    int chain_gx, chain_gy; // tiles per image (chain_gx * chain_gy workgroups per image)
    int chain_tab;          // byte offset of the ChainRect table ([tile][level]) in ltab
    int chain_toffs;        // byte offset of the per-tile table offsets ([tile][level + 1] ints)
    int chain_buf;          // LDS bytes of one level buffer (two, ping-pong)
    int chain_rs;           // LDS bytes of the blur row sums
    int chain_lds;          // total dynamic LDS of the launch
    LevelGeom lv[ORBX_MAX_LEVELS];
};

// k_fast ROI row pitch in dwords: a multiple of 4 (16-byte aligned rows for the
// compass's b128 reads) with room for the widest lane's reads (16 pixels per lane, 2 lanes
// per detection row up to 32 columns, else 4).  A bank-conflict-free pitch (24 / 48 dwords)
// was measured slower: the larger ROI costs a workgroup per CU.
#define FAST_NC 4        // k_fast cells per wave at large batches (the next cell's ROI loads
                         // overlap this cell's work); small batches take fewer
#define FAST_PF2D 10     // its rows per lane: ROIs up to 40 rows are prefetched
__host__ __device__ inline int fast_lpitch(int ndw, int dw) {
    const int lpr = dw > 32 ? 4 : 2;
    const int need = ndw > 4 * lpr + 4 ? ndw : 4 * lpr + 4;
    return (need + 3) & ~3;
}

// Packed candidate / octree survivor: x, y relative to (minBorderX, minBorderY).
__host__ __device__ inline uint32_t pack_cand(int x, int y, int score) {
    return (uint32_t)x | ((uint32_t)y << 12) | ((uint32_t)score << 24);
}
__host__ __device__ inline int cand_x(uint32_t c) { return (int)(c & 0xFFF); }
__host__ __device__ inline int cand_y(uint32_t c) { return (int)((c >> 12) & 0xFFF); }
__host__ __device__ inline int cand_s(uint32_t c) { return (int)(c >> 24); }

}  // namespace orbx
