// ffd_haar.hip — gfx950 Haar face detector: FaceForest::detectFace (src/FaceForest.cpp:136-159),
// i.e. OpenCV 2.4.9 CascadeClassifier::detectMultiScale(frame, boxes, 1.3, 1, 0, Size(30, 30)) on the
// new-format stump cascade data/haarcascade_frontalface_alt.xml, then detectFace's widening.
// Bit-exact with the CPU restatement oracle/ffd_oracle.cpp (haar_scan / haar_group / widen_box),
// which states the OpenCV semantics followed (parity with OpenCV itself unpinned: no OpenCV here).
//
// A batch of frames runs as one pass of six launches over a host-built level table (one level per
// (frame, pyramid scale) that detectMultiScale scans):
//   k_haar_gray      cvtColor(BGR2GRAY) of each frame, once per frame
//   k_haar_resize    the pyramid level: resize(INTER_LINEAR) to cvRound(cols / f) x cvRound(rows / f)
//   k_haar_rows      per level row: u32 prefix sums of v and v^2 (a wave per row, DPP scans)
//   k_haar_cols      per level column: the running column sums -> integral sum (i32) / sqsum (u64)
//   k_haar_cascade   a thread per scan position (x, y on the yStep grid): predictOrderedStump over the
//                    22 stages, weak classifiers read as wave-uniform scalar loads; result per position
//   k_haar_collect   a workgroup per frame: each thread walks one scan row applying the invoker's
//                    skip rule (a stage-0 reject skips the next x) and emits the candidates in scan
//                    order (block prefix sums)
//   k_haar_group     a workgroup per frame: groupRectangles (connected components of SimilarRects by
//                    min-label propagation = cv::partition's classes, numbered by smallest member),
//                    averages, the small-inside-large filter, detectFace's widening + intersect
// Integer-exact integrals (sum < 2^31, sqsum < 2^53 as u64), fp32 / fp64 evaluated in the
// restatement's operation order (-ffp-contract=off), so every position's result is identical.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "ffd_haar.hpp"

namespace ffd {

namespace {

__device__ __forceinline__ int hsat_u8(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }
__device__ __forceinline__ int hsat_s16(int v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }
__device__ __forceinline__ int hround(float v) {  // cvRound(float)
  if (!(v >= -2147483648.0f && v < 2147483648.0f)) return (int)0x80000000;
  return (int)__builtin_rintf(v);
}
__device__ __forceinline__ int hround_d(double v) {  // cvRound(double)
  if (!(v >= -2147483648.0 && v < 2147483648.0)) return (int)0x80000000;
  return (int)__builtin_rint(v);
}

// inclusive prefix sum over a wave (DPP row shifts + row broadcasts); integer adds
__device__ __forceinline__ uint32_t wave_scan_u32(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);
  return v;
}

// ---------------------------------------------------------------------------- gray ----
__global__ __launch_bounds__(256) void k_haar_gray(const HaarFrame* __restrict__ frames,
                                                   const uint8_t* __restrict__ images, uint8_t* __restrict__ gray) {
  const HaarFrame f = frames[blockIdx.y];
  const uint8_t* img = images + f.img_off;
  uint8_t* g = gray + f.gray_off;
  const int cpr = (f.w + 255) / 256, n = cpr * f.h;  // steps of 256 pixels of one row (the row index wave-uniform)
  for (int t = blockIdx.x; t < n; t += gridDim.x) {
    const int y = t / cpr, x = (t - y * cpr) * 256 + threadIdx.x;
    if (x >= f.w) continue;
    const uint8_t* p = img + (int64_t)y * f.stride + 3 * x;
    g[(int64_t)y * f.w + x] = (uint8_t)((p[0] * 1868 + p[1] * 9617 + p[2] * 4899 + (1 << 13)) >> 14);
  }
}

// ------------------------------------------------------------------------ resize ----
// resize(INTER_LINEAR) 8U as oracle cv_resize (OpenCV 2.4.9 fixed point: 11-bit horizontal
// coefficients, SSE2 vertical pass on columns [0, xv), scalar tail); mode 0 copy, 2 area 2x.
// A workgroup step is a tile of 256 columns x HZ_ROWS rows: each thread's column coefficients (source column,
// 11-bit weights) are computed once for the tile's rows, each row's (wave-uniform) once per row — the same
// expressions as per pixel, hoisted (round 6: a thread per pixel with an integer division and both coefficient sets
// per pixel, C3 377 us per 64 frames).
#ifndef FFD_HAAR_RESIZE_ROWS
#define FFD_HAAR_RESIZE_ROWS 8
#endif
constexpr int HZ_ROWS = FFD_HAAR_RESIZE_ROWS;
__global__ __launch_bounds__(256) void k_haar_resize(const HaarLevel* __restrict__ levels,
                                                     const uint8_t* __restrict__ gray, uint8_t* __restrict__ scaled) {
  const HaarLevel L = levels[blockIdx.y];
  const uint8_t* src = gray + L.gray_off;
  uint8_t* dst = scaled + L.img_off;
  const int sw = L.src_w, sh = L.src_h;
  const int ncb = (L.sw + 255) / 256, tiles = ncb * ((L.sh + HZ_ROWS - 1) / HZ_ROWS);
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int rb = t / ncb, dx = (t - rb * ncb) * 256 + threadIdx.x, y0 = rb * HZ_ROWS, y1 = min(L.sh, y0 + HZ_ROWS);
    if (dx >= L.sw) continue;
    uint8_t* out = dst + (int64_t)y0 * L.sw + dx;
    if (L.mode == 0) {
      for (int dy = y0; dy < y1; dy++, out += L.sw) *out = src[(int64_t)dy * sw + dx];
      continue;
    }
    if (L.mode == 2) {
      for (int dy = y0; dy < y1; dy++, out += L.sw) {
        const uint8_t* s0 = src + (int64_t)(2 * dy) * sw + 2 * dx;
        *out = (uint8_t)((s0[0] + s0[1] + s0[sw] + s0[sw + 1] + 2) >> 2);
      }
      continue;
    }
    float fx = (float)((dx + 0.5) * L.scale_x - 0.5);
    int sx = (int)floorf(fx);
    fx -= sx;
    if (sx < 0) fx = 0, sx = 0;
    bool right = false;
    if (sx + 1 >= sw) {
      right = true;
      if (sx >= sw - 1) fx = 0, sx = sw - 1;
    }
    const int a0 = right ? 2048 : hsat_s16(hround((1.f - fx) * 2048.f)), a1 = right ? 0 : hsat_s16(hround(fx * 2048.f));
    const int sx1 = right ? sx : sx + 1;  // (right: r = p[sx] * 2048, as a0 = 2048, a1 = 0 gives)
    const bool vec = dx < L.xv;
    for (int dy = y0; dy < y1; dy++, out += L.sw) {
      float fy = (float)((dy + 0.5) * L.scale_y - 0.5);
      const int sy = (int)floorf(fy);
      fy -= sy;
      const int b0 = hsat_s16(hround((1.f - fy) * 2048.f)), b1 = hsat_s16(hround(fy * 2048.f));
      const int yy0 = min(max(sy, 0), sh - 1), yy1 = min(max(sy + 1, 0), sh - 1);
      const uint8_t* r0p = src + (int64_t)yy0 * sw;
      const uint8_t* r1p = src + (int64_t)yy1 * sw;
      const int r0 = r0p[sx] * a0 + r0p[sx1] * a1, r1 = r1p[sx] * a0 + r1p[sx1] * a1;
      int v;
      if (vec) {
        const int s0 = max(-32768, min(32767, r0 >> 4)), s1 = max(-32768, min(32767, r1 >> 4));
        int m = max(-32768, min(32767, ((s0 * b0) >> 16) + ((s1 * b1) >> 16)));
        m = max(-32768, min(32767, m + 2)) >> 2;
        v = hsat_u8(m);
      } else {
        v = hsat_u8((b0 * r0 + b1 * r1 + (1 << 21)) >> 22);
      }
      *out = (uint8_t)v;
    }
  }
}

// ---------------------------------------------------------------------- integrals ----
// Pass 1: one wave per (level, row y): prefix sums of v and v*v along the row into sum[y + 1][x + 1] / sq[y + 1][x + 1];
// column 0 and row 0 are zeroed here.  The squared integral is kept modulo 2^32 (u32): the cascade only reads it
// through the normrect's four-corner sum, whose true value is below 2^32 (ffd_detect.cpp checks the window), so the
// modular difference is exact — half the bytes of a u64 plane in both passes and the cascade's corner reads.
__global__ __launch_bounds__(256) void k_haar_rows(const HaarLevel* __restrict__ levels,
                                                   const uint8_t* __restrict__ scaled, int32_t* __restrict__ sum,
                                                   uint32_t* __restrict__ sq) {
  const HaarLevel L = levels[blockIdx.y];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int P = L.sw + 1;
  int32_t* S = sum + L.sum_off;
  uint32_t* Q = sq + L.sum_off;
  for (int y = blockIdx.x * 4 + wv; y <= L.sh; y += gridDim.x * 4) {
    if (y == 0) {
      for (int x = lane; x < P; x += 64) { S[x] = 0; Q[x] = 0; }
      continue;
    }
    const uint8_t* row = scaled + L.img_off + (int64_t)(y - 1) * L.sw;
    int32_t* so = S + (int64_t)y * P;
    uint32_t* qo = Q + (int64_t)y * P;
    if (lane == 0) { so[0] = 0; qo[0] = 0; }
    uint32_t cs = 0, cq = 0;
    for (int x0 = 0; x0 < L.sw; x0 += 64) {
      const int x = x0 + lane;
      const uint32_t v = x < L.sw ? row[x] : 0u;
      const uint32_t ps = wave_scan_u32(v), pq = wave_scan_u32(v * v);
      if (x < L.sw) { so[x + 1] = (int32_t)(cs + ps); qo[x + 1] = cq + pq; }
      cs += (uint32_t)__builtin_amdgcn_readlane((int)ps, 63);
      cq += (uint32_t)__builtin_amdgcn_readlane((int)pq, 63);
    }
  }
}

// Pass 2: one thread per (level, column x >= 1): running sums down the rows, FFD_HAAR_COLS_RIF rows' loads in
// flight (the kernel lasts as long as the tallest level's column chain).
#ifndef FFD_HAAR_COLS_RIF
#define FFD_HAAR_COLS_RIF 32  // (C3 detection 77.9 -> 76.6 ms per 512 frames against 8)
#endif
__global__ __launch_bounds__(256) void k_haar_cols(const HaarLevel* __restrict__ levels, int32_t* __restrict__ sum,
                                                   uint32_t* __restrict__ sq) {
  constexpr int R = FFD_HAAR_COLS_RIF;
  const HaarLevel L = levels[blockIdx.y];
  const int x = 1 + blockIdx.x * 256 + threadIdx.x;
  if (x > L.sw) return;
  const int P = L.sw + 1;
  int32_t* S = sum + L.sum_off + x;
  uint32_t* Q = sq + L.sum_off + x;
  int32_t as = 0;
  uint32_t aq = 0;
  for (int y0 = 1; y0 <= L.sh; y0 += R) {
    int32_t vs[R];
    uint32_t vq[R];
#pragma unroll
    for (int k = 0; k < R; k++)
      if (y0 + k <= L.sh) { vs[k] = S[(int64_t)(y0 + k) * P]; vq[k] = Q[(int64_t)(y0 + k) * P]; }
#pragma unroll
    for (int k = 0; k < R; k++)
      if (y0 + k <= L.sh) {
        as += vs[k];
        aq += vq[k];
        S[(int64_t)(y0 + k) * P] = as;
        Q[(int64_t)(y0 + k) * P] = aq;
      }
  }
}

// ------------------------------------------------------------------------ cascade ----
// predictOrderedStump for a tile of 64 x 8 scan positions per workgroup.  The tile's integral
// window (sum, i32) is staged once in LDS, so every rectangle corner is an LDS read; the squared
// integral is read from HBM only for the 4 normrect corners.  The tile's positions then run the
// stages in passes ([0,1), [1,2), [2,4), [4,7), [7,n)): between passes the survivors are compacted
// into an LDS list, so the waves of later passes are dense (without it almost every wave keeps some
// lane alive through the early stages and runs ~100 weak classifiers for lanes that need ~10).
// Each stage's sum restarts at 0, so splitting at stage boundaries is exact.
// Result per position: 1 (face) or -stage (stage 0 -> 0), as int8.
#ifndef FFD_HAAR_GROUP_LANES
#define FFD_HAAR_GROUP_LANES 8  // lanes per survivor in the last FFD_HAAR_GROUP_PASSES passes (1: a lane each)
#endif
#ifndef FFD_HAAR_GROUP_PASSES
#define FFD_HAAR_GROUP_PASSES 1
#endif
#ifndef FFD_HAAR_BATCH2
#define FFD_HAAR_BATCH2 2  // two-rectangle classifiers evaluated per step (their corner reads issued together)
#endif
#ifndef FFD_HAAR_BATCH3
#define FFD_HAAR_BATCH3 2  // three-rectangle classifiers per step (2 / 2: 58 VGPRs, C3 detection 83.7 -> 81.3 ms; 4 / 4: 84)
#endif
#ifndef FFD_HAAR_THREADS
#define FFD_HAAR_THREADS 256
#endif
constexpr int HT_X = 64, HT_Y = FFD_HAAR_TILE_Y, HT_THREADS = FFD_HAAR_THREADS, HT_POS = HT_X * HT_Y;
#ifndef FFD_HAAR_PASSES
#define FFD_HAAR_PASSES 5  // survivor-compaction passes over the stages (5: [0,1) [1,2) [2,4) [4,7) [7,n))
#endif

static_assert(HT_X == HAAR_TILE_X && HT_Y == HAAR_TILE_Y, "host offset tables assume this tile");
__host__ __device__ constexpr int haar_win_cols(int ystep, int ww) { return HT_X * ystep + ww; }
__host__ __device__ constexpr int haar_win_rows(int ystep, int wh) { return HT_Y * ystep + wh; }

__global__ __launch_bounds__(HT_THREADS) void k_haar_cascade(const HaarLevel* __restrict__ levels, int n_levels,
                                                             const int32_t* __restrict__ sum,
                                                             const uint32_t* __restrict__ sq,
                                                             const HaarWeak* __restrict__ weak_tables, int n_weak,
                                                             const HaarStage* __restrict__ stages, int n_stages,
                                                             int ww, int wh, int order_free,
                                                             int8_t* __restrict__ result) {
  extern __shared__ __attribute__((aligned(16))) int32_t win[];
  __shared__ double vnf[HT_POS];
  __shared__ uint16_t list[2][HT_POS];
  __shared__ int n_list[2];
  // this workgroup's level: the last whose first tile is <= blockIdx.x (the grid holds every level's tiles and
  // nothing else; a (tile, level) grid over the largest level's tile count launched ~6x as many empty workgroups)
  int lo = 0, hi = n_levels - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (levels[mid].tile0 <= (int)blockIdx.x) lo = mid;
    else hi = mid - 1;
  }
  const HaarLevel L = levels[lo];
  const int tiles_x = (L.nx + HT_X - 1) / HT_X, tl = (int)blockIdx.x - L.tile0;
  const int ty = tl / tiles_x, tx = tl - ty * tiles_x;
  if (ty * HT_Y >= L.ny) return;
  const int ys = L.ystep, P = L.sw + 1;
  const int WC = haar_win_cols(ys, ww), WR = haar_win_rows(ys, wh);
  const int x0 = tx * HT_X * ys, y0 = ty * HT_Y * ys;
  const HaarWeak* __restrict__ weak = weak_tables + (ys == 2 ? n_weak : 0);  // offsets for this window pitch
  const int32_t* S = sum + L.sum_off;
  const uint32_t* Q = sq + L.sum_off;
  // setWindow for every position of the tile: normrect (1, 1, ww - 2, wh - 2)
  const int na = haar_window_offset(ys, WC, 1, 1), nb = haar_window_offset(ys, WC, 1, ww - 1);
  const int nc = haar_window_offset(ys, WC, wh - 1, 1), nd = haar_window_offset(ys, WC, wh - 1, ww - 1);
  for (int i = threadIdx.x; i < WC * WR; i += HT_THREADS) {
    const int r = i / WC, c = i - r * WC;
    const int gy = y0 + r, gx = x0 + c;
    win[haar_window_offset(ys, WC, r, c)] = (gy <= L.sh && gx < P) ? S[(int64_t)gy * P + gx] : 0;
  }
  if (threadIdx.x == 0) { n_list[0] = 0; n_list[1] = 0; }
  __syncthreads();
  const int qa = P + 1, qb = qa + (ww - 2), qc = (wh - 1) * P + 1, qd = qc + (ww - 2);
  for (int p = threadIdx.x; p < HT_POS; p += HT_THREADS) {
    const int lx = p & (HT_X - 1), ly = p / HT_X;
    const int ix = tx * HT_X + lx, iy = ty * HT_Y + ly;
    if (ix >= L.nx || iy >= L.ny) continue;
    const int o = ly * ys * WC + lx;  // window(ys ly, ys lx): see haar_window_offset
    const int valsum = win[o + na] - win[o + nb] - win[o + nc] + win[o + nd];
    const uint32_t* q = Q + (int64_t)(y0 + ly * ys) * P + x0 + lx * ys;
    const double valsq = (double)(uint32_t)(q[qa] - q[qb] - q[qc] + q[qd]);  // (exact modulo 2^32, see k_haar_rows)
    double nf = (double)((ww - 2) * (wh - 2)) * valsq - (double)valsum * (double)valsum;
    nf = nf > 0. ? __builtin_sqrt(nf) : 1.;
    vnf[p] = 1. / nf;
    list[0][atomicAdd(&n_list[0], 1)] = (uint16_t)p;  // order within a pass does not matter
  }
  __syncthreads();
#if FFD_HAAR_PASSES == 8
  constexpr int NP = 8;
  const int bounds[NP + 1] = {0, 1, 2, 4, 7, 10, 13, 17, n_stages};
#else
  constexpr int NP = 5;
  const int bounds[NP + 1] = {0, 1, 2, 4, 7, n_stages};
#endif
  int cur = 0;
  for (int pass = 0; pass < NP; pass++) {
    const int s0 = min(bounds[pass], n_stages), s1 = pass == NP - 1 ? n_stages : min(bounds[pass + 1], n_stages);
    if (s0 >= s1) continue;
    const int n = n_list[cur];
    if (threadIdx.x == 0) n_list[cur ^ 1] = 0;
    __syncthreads();
#if FFD_HAAR_GROUP_LANES > 1
    if (order_free && pass >= NP - FFD_HAAR_GROUP_PASSES) {
      // Sparse late passes: FFD_HAAR_GROUP_LANES lanes per survivor, each summing every G-th classifier
      // of a stage (records as vector loads), the partial sums combined across the group.  Valid
      // because the host proved every stage's double leaf sum exact in any order (order_free).
      constexpr int G = FFD_HAAR_GROUP_LANES;
      const int sub = threadIdx.x & (G - 1);
      for (int k = threadIdx.x / G; k < n; k += HT_THREADS / G) {
        const int p = list[cur][k];
        const int lx = p & (HT_X - 1), ly = p / HT_X;
        const int32_t* w0 = win + ly * ys * WC + lx;
        const double f = vnf[p];
        auto rs = [&](uint32_t ab, uint32_t cd) {
          return w0[ab & 0xFFFFu] - w0[ab >> 16] - w0[cd & 0xFFFFu] + w0[cd >> 16];
        };
        int s = s0;
        for (; s < s1; s++) {
          const HaarStage st = stages[s];
          double acc = 0.0;
          const int e = st.first + st.ntrees;
          for (int i = st.first + sub; i < e; i += G) {
            const HaarWeak c = weak[i];
            float ret;
            if (c.o[3] == HAAR_SHARED) {  // (ffd_haar.hpp)
              const int e = w0[c.o[0] & 0xFFFFu] - w0[c.o[0] >> 16];
              ret = c.w0 * (float)(e - w0[c.o[1] & 0xFFFFu] + w0[c.o[1] >> 16]) +
                    c.w1 * (float)(e - w0[c.o[2] & 0xFFFFu] + w0[c.o[2] >> 16]);
            } else {
              ret = c.w0 * (float)rs(c.o[0], c.o[1]) + c.w1 * (float)rs(c.o[2], c.o[3]);
              if (c.w2 != 0.0f) ret += c.w2 * (float)rs(c.o[4], c.o[5]);  // rect 2 empty: + 0 (see above)
            }
            const double v = (double)ret * f;
            acc += (double)(v < (double)c.thr ? c.leaf0 : c.leaf1);
          }
#pragma unroll
          for (int d = 1; d < G; d <<= 1) acc += __shfl_xor(acc, d);
          if (acc < (double)st.thr) break;
        }
        if (sub == 0) {
          const int ix = tx * HT_X + lx, iy = ty * HT_Y + ly;
          if (s < s1) result[L.res_off + (int64_t)iy * L.nx + ix] = (int8_t)(-s);
          else if (s1 == n_stages) result[L.res_off + (int64_t)iy * L.nx + ix] = 1;
          else list[cur ^ 1][atomicAdd(&n_list[cur ^ 1], 1)] = (uint16_t)p;
        }
      }
      __syncthreads();
      cur ^= 1;
      continue;
    }
#endif
#ifdef FFD_HAAR_PROBE_SKIPFROM  // timing probe only (wrong results): passes >= this reject without evaluating
    if (pass >= FFD_HAAR_PROBE_SKIPFROM) {
      for (int k = threadIdx.x; k < n; k += HT_THREADS) {
        const int p = list[cur][k];
        const int ix = tx * HT_X + (p & (HT_X - 1)), iy = ty * HT_Y + p / HT_X;
        result[L.res_off + (int64_t)iy * L.nx + ix] = (int8_t)(-s0);
      }
      break;
    }
#endif
    for (int k = threadIdx.x; k < n; k += HT_THREADS) {
      const int p = list[cur][k];
      const int lx = p & (HT_X - 1), ly = p / HT_X;
      const int32_t* w0 = win + ly * ys * WC + lx;
      const double f = vnf[p];
      int s = s0;
      for (; s < s1; s++) {
        const HaarStage st = stages[s];
        double acc = 0.0;
        // 4 weak classifiers per step: their records (wave-uniform scalar loads) and all window reads
        // are issued together; the sum accumulates in record order (two-rectangle classifiers first:
        // the host checked that this stage's sum is exact in any order, HaarStage::n_two)
        auto rs = [&](uint32_t ab, uint32_t cd) {  // corner offsets precomputed for this window pitch
          return w0[ab & 0xFFFFu] - w0[ab >> 16] - w0[cd & 0xFFFFu] + w0[cd >> 16];
        };
        // kind: 0 two rectangles, 1 three, 2 two sharing two corners (HAAR_SHARED: six corner reads)
        auto value_of = [&](const HaarWeak& c, auto kind) {
          float ret;
          if constexpr (decltype(kind)::value == 2) {
            const int e = w0[c.o[0] & 0xFFFFu] - w0[c.o[0] >> 16];
            ret = c.w0 * (float)(e - w0[c.o[1] & 0xFFFFu] + w0[c.o[1] >> 16]) +
                  c.w1 * (float)(e - w0[c.o[2] & 0xFFFFu] + w0[c.o[2] >> 16]);
          } else {
            ret = c.w0 * (float)rs(c.o[0], c.o[1]) + c.w1 * (float)rs(c.o[2], c.o[3]);
            if constexpr (decltype(kind)::value == 1) ret += c.w2 * (float)rs(c.o[4], c.o[5]);
          }
          // HaarEvaluator::operator() (cascadedetect.hpp, 2.4.9) returns double: calc() * varianceNormFactor,
          // compared unrounded with the float threshold in predictOrderedStump
          return (double)ret * f;
        };
        auto run = [&](int i, int e, auto kind) {
          constexpr int NB = decltype(kind)::value == 1 ? FFD_HAAR_BATCH3 : FFD_HAAR_BATCH2;
          for (; i + NB <= e; i += NB) {
            HaarWeak c[NB];
            double v[NB];
#pragma unroll
            for (int j = 0; j < NB; j++) c[j] = weak[i + j];
#pragma unroll
            for (int j = 0; j < NB; j++) v[j] = value_of(c[j], kind);
#pragma unroll
            for (int j = 0; j < NB; j++) acc += (double)(v[j] < (double)c[j].thr ? c[j].leaf0 : c[j].leaf1);
          }
          for (; i < e; i++) {
            const HaarWeak c = weak[i];
            const double v = value_of(c, kind);
            acc += (double)(v < (double)c.thr ? c.leaf0 : c.leaf1);
          }
        };
        // two-rectangle features: rect 2 is empty (w2 = 0), and + 0 * 0 leaves ret unchanged up to the
        // sign of a zero, which no comparison distinguishes
        run(st.first, st.first + st.n_sh, std::integral_constant<int, 2>{});
        run(st.first + st.n_sh, st.first + st.n_two, std::integral_constant<int, 0>{});
        run(st.first + st.n_two, st.first + st.ntrees, std::integral_constant<int, 1>{});
        if (acc < (double)st.thr) break;
      }
      const int ix = tx * HT_X + lx, iy = ty * HT_Y + ly;
      if (s < s1) result[L.res_off + (int64_t)iy * L.nx + ix] = (int8_t)(-s);
      else if (s1 == n_stages) result[L.res_off + (int64_t)iy * L.nx + ix] = 1;
      else list[cur ^ 1][atomicAdd(&n_list[cur ^ 1], 1)] = (uint16_t)p;
    }
    __syncthreads();
    cur ^= 1;
  }
}

// ------------------------------------------------------------------------ collect ----
constexpr int HC_THREADS = 1024;
#ifndef FFD_HAAR_COLLECT_SERIAL
#define FFD_HAAR_COLLECT_SERIAL 0  // 1: the thread-per-row scan (k_haar_collect)
#endif

__device__ __forceinline__ int block_excl_scan(int v, int* sh, int& total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int incl = (int)wave_scan_u32((uint32_t)v);
  if (lane == 63) sh[wv] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int w = 0; w < HC_THREADS / 64; w++) { int t = sh[w]; sh[w] = acc; acc += t; }
    sh[HC_THREADS / 64] = acc;
  }
  __syncthreads();
  const int r = sh[wv] + incl - v;
  total = sh[HC_THREADS / 64];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(HC_THREADS) void k_haar_collect(const HaarFrame* __restrict__ frames,
                                                              const HaarLevel* __restrict__ levels,
                                                              const int8_t* __restrict__ result, int cap,
                                                              int4* __restrict__ cand, int32_t* __restrict__ n_cand) {
  __shared__ int sh[HC_THREADS / 64 + 1];
  const HaarFrame f = frames[blockIdx.x];
  int base = 0;
  for (int r0 = 0; r0 < f.rows; r0 += HC_THREADS) {
    const int r = r0 + threadIdx.x;
    int lv = -1, iy = 0;
    if (r < f.rows) {
      lv = f.level0;
      while (lv + 1 < f.level1 && levels[lv + 1].row0 <= r) lv++;
      iy = r - levels[lv].row0;
    }
    // invoker scan of one row: x steps by yStep, a stage-0 reject (result 0) skips the next x
    auto walk = [&](bool emit, int at) {
      int n = 0;
      if (lv < 0) return 0;
      const HaarLevel& L = levels[lv];
      const int8_t* row = result + L.res_off + (int64_t)iy * L.nx;
      // 16 results per batch of independent loads, so the skip chain runs in registers instead of
      // one dependent load per step
      int ix = 0;
      for (int c0 = 0; c0 < L.nx; c0 += 16) {
        int8_t v16[16];
#pragma unroll
        for (int k = 0; k < 16; k++) v16[k] = c0 + k < L.nx ? row[c0 + k] : (int8_t)-1;
#pragma unroll
        for (int k = 0; k < 16; k++) {
          if (ix != c0 + k) continue;
          const int v = v16[k];
          if (c0 + k >= L.nx) break;
          if (v > 0) {
            if (emit && at + n < cap) {
              const int x = ix * L.ystep, y = iy * L.ystep;
              cand[(int64_t)blockIdx.x * cap + at + n] =
                  make_int4(hround_d(x * L.factor), hround_d(y * L.factor), L.win_w, L.win_h);
            }
            n++;
          }
          ix += v == 0 ? 2 : 1;
        }
      }
      return n;
    };
    const int cnt = walk(false, 0);
    int tot;
    const int off = block_excl_scan(cnt, sh, tot);
    walk(true, base + off);
    base += tot;
  }
  if (threadIdx.x == 0) n_cand[blockIdx.x] = base;
}

// Default form of the same scan, spread over (frame, block of HR_THREADS rows) workgroups: the
// per-frame form above runs one workgroup per frame (64 per group of frames, a quarter of the CUs).
// k_haar_rowcount counts each row's candidates (a wave per row; only a row holding a face is walked); k_haar_emit sums the counts of the
// frame's earlier rows, scans its own and walks again, writing each candidate at its slot.  Same
// walk, same candidate order, same cap rule.
constexpr int HR_THREADS = 256;

__device__ __forceinline__ int haar_row_walk(const HaarFrame& f, const HaarLevel* __restrict__ levels,
                                             const int8_t* __restrict__ result, int r, bool emit, int at, int cap,
                                             int4* __restrict__ out) {
  int lv = f.level0;
  while (lv + 1 < f.level1 && levels[lv + 1].row0 <= r) lv++;
  const HaarLevel& L = levels[lv];
  const int iy = r - L.row0;
  const int8_t* row = result + L.res_off + (int64_t)iy * L.nx;
  int n = 0, ix = 0;
  for (int c0 = 0; c0 < L.nx; c0 += 16) {
    int8_t v16[16];
#pragma unroll
    for (int k = 0; k < 16; k++) v16[k] = c0 + k < L.nx ? row[c0 + k] : (int8_t)-1;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      if (ix != c0 + k) continue;
      const int v = v16[k];
      if (c0 + k >= L.nx) break;
      if (v > 0) {
        if (emit && at + n < cap) {
          const int x = ix * L.ystep, y = iy * L.ystep;
          out[at + n] = make_int4(hround_d(x * L.factor), hround_d(y * L.factor), L.win_w, L.win_h);
        }
        n++;
      }
      ix += v == 0 ? 2 : 1;
    }
  }
  return n;
}

__global__ __launch_bounds__(HR_THREADS) void k_haar_rowcount(const HaarFrame* __restrict__ frames,
                                                               const HaarLevel* __restrict__ levels,
                                                               const int8_t* __restrict__ result, int pitch,
                                                               int32_t* __restrict__ rowcnt) {
  // a wave per scan row: the row's results read coalesced, walked (by lane 0) only when it holds a face — most rows
  // hold none (round 5: a thread per row walking every row, C3 detection 77.1 -> 75.6 ms per 512 frames)
  const HaarFrame f = frames[blockIdx.x];
  const int lane = threadIdx.x & 63, r = blockIdx.y * (HR_THREADS / 64) + (threadIdx.x >> 6);
  if (r >= f.rows) return;  // whole wave
  int lv = f.level0;
  while (lv + 1 < f.level1 && levels[lv + 1].row0 <= r) lv++;
  const HaarLevel& L = levels[lv];
  const int8_t* row = result + L.res_off + (int64_t)(r - L.row0) * L.nx;
  bool face = false;
  for (int c = lane; c < L.nx; c += 64) face |= row[c] > 0;
  if (__ballot(face) == 0ull) {  // no face in the row: the walk counts nothing
    if (lane == 0) rowcnt[(int64_t)blockIdx.x * pitch + r] = 0;
    return;
  }
  if (lane == 0) rowcnt[(int64_t)blockIdx.x * pitch + r] = haar_row_walk(f, levels, result, r, false, 0, 0, nullptr);
}

__global__ __launch_bounds__(HR_THREADS) void k_haar_emit(const HaarFrame* __restrict__ frames,
                                                           const HaarLevel* __restrict__ levels,
                                                           const int8_t* __restrict__ result, int pitch,
                                                           const int32_t* __restrict__ rowcnt, int cap,
                                                           int4* __restrict__ cand, int32_t* __restrict__ n_cand) {
  __shared__ int sh[HR_THREADS / 64 + 1];
  const HaarFrame f = frames[blockIdx.x];
  const int r0 = blockIdx.y * HR_THREADS;
  if (r0 >= f.rows && !(r0 == 0 && f.rows == 0)) return;  // whole workgroup
  const int32_t* rc = rowcnt + (int64_t)blockIdx.x * pitch;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int before = 0;
  for (int i = threadIdx.x; i < r0; i += HR_THREADS) before += rc[i];
  before = __shfl((int)wave_scan_u32((uint32_t)before), 63);
  if (lane == 0) sh[wv] = before;
  __syncthreads();
  before = 0;
#pragma unroll
  for (int w = 0; w < HR_THREADS / 64; w++) before += sh[w];
  __syncthreads();
  const int r = r0 + threadIdx.x;
  const int cnt = r < f.rows ? rc[r] : 0;
  const int incl = (int)wave_scan_u32((uint32_t)cnt);
  if (lane == 63) sh[wv] = incl;
  __syncthreads();
  int off = before + incl - cnt, tot = before;
#pragma unroll
  for (int w = 0; w < HR_THREADS / 64; w++) {
    off += w < wv ? sh[w] : 0;
    tot += sh[w];
  }
  if (cnt > 0) (void)haar_row_walk(f, levels, result, r, true, off, cap, cand + (int64_t)blockIdx.x * cap);
  if (threadIdx.x == 0 && (f.rows == 0 || blockIdx.y == (f.rows - 1) / HR_THREADS)) n_cand[blockIdx.x] = tot;
}

// -------------------------------------------------------------------------- group ----
__device__ __forceinline__ bool similar_rects(int4 a, int4 b, double eps) {  // cv::SimilarRects
  const double delta = eps * (double)(min(a.z, b.z) + min(a.w, b.w)) * 0.5;
  return (double)abs(a.x - b.x) <= delta && (double)abs(a.y - b.y) <= delta &&
         (double)abs(a.x + a.z - b.x - b.z) <= delta && (double)abs(a.y + a.w - b.y - b.w) <= delta;
}

__device__ __forceinline__ int ld_agent(const int* p) {  // coherent read of a value other waves wrote atomically
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// GLOBAL: the component labels in global memory (label_g, cap per frame) for frames with more raw candidates
// than the LDS holds (HAAR_MAX_CAND); the same algorithm, the labels read and written with relaxed atomics.
template <bool GLOBAL>
__global__ __launch_bounds__(HC_THREADS) void k_haar_group(const HaarFrame* __restrict__ frames, int cap,
                                                            const int4* __restrict__ cand,
                                                            const int32_t* __restrict__ n_cand, int min_neighbors,
                                                            int widen, int4* __restrict__ cls_rect,
                                                            int* __restrict__ cls_sum, int4* __restrict__ boxes,
                                                            int32_t* __restrict__ n_boxes, int* __restrict__ label_g) {
  // (GLOBAL: the labels arrive converged from k_haar_label_round / k_haar_label_jump, spread over the chip)
  __shared__ int label_s[GLOBAL ? 1 : HAAR_MAX_CAND];
  int* const labp = GLOBAL ? label_g + (int64_t)blockIdx.x * cap : label_s;
  auto lget = [&](int i) -> int {
    if constexpr (GLOBAL) return __hip_atomic_load(labp + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return labp[i];
  };
  auto lset = [&](int i, int v) {
    if constexpr (GLOBAL) __hip_atomic_store(labp + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else labp[i] = v;
  };
  __shared__ int sh[HC_THREADS / 64 + 1];
  __shared__ int changed;
  const HaarFrame f = frames[blockIdx.x];
  const int N = min(n_cand[blockIdx.x], cap);
  const int4* R = cand + (int64_t)blockIdx.x * cap;
  int4* out = boxes + (int64_t)blockIdx.x * cap;
  const double eps = 0.2;  // detectMultiScale GROUP_EPS
  if (min_neighbors <= 0) {  // groupRectangles returns the list unchanged
    for (int i = threadIdx.x; i < N; i += HC_THREADS) out[i] = R[i];
    if (threadIdx.x == 0) n_boxes[blockIdx.x] = N;
    return;
  }
  // connected components of SimilarRects: every label converges to its component's smallest index
  if (!GLOBAL) for (int i = threadIdx.x; i < N; i += HC_THREADS) lset(i, i);
  for (; !GLOBAL;) {
    if (threadIdx.x == 0) changed = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < N; i += HC_THREADS) {
      const int4 ri = R[i];
      int m = lget(i);
      for (int j = 0; j < N; j++)
        if (j != i && lget(j) < m && similar_rects(ri, R[j], eps)) m = lget(j);
      if (m < lget(i)) { lset(i, m); changed = 1; }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < N; i += HC_THREADS) {  // pointer jumping (labels only decrease)
      int l = lget(i);
      while (lget(l) != l) l = lget(l);
      lset(i, l);
    }
    __syncthreads();
    if (!changed) break;
    __syncthreads();
  }
  // class ids in order of their smallest member (cv::partition's numbering)
  int* csum = cls_sum + (int64_t)blockIdx.x * cap * 5;  // per class: x, y, w, h sums, count
  int ncls = 0;
  for (int i0 = 0; i0 < N; i0 += HC_THREADS) {
    const int i = i0 + threadIdx.x;
    const int is_root = (i < N && lget(i) == i) ? 1 : 0;
    int tot;
    const int id = block_excl_scan(is_root, sh, tot) + ncls;
    if (is_root) {
      lset(i, -1 - id);  // roots now hold ~class id (members still point at the root index)
      for (int k = 0; k < 5; k++) __hip_atomic_store(&csum[id * 5 + k], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    ncls += tot;
  }
  __threadfence();
  __syncthreads();
  for (int i = threadIdx.x; i < N; i += HC_THREADS) {
    const int l = lget(i);
    const int id = l < 0 ? -1 - l : -1 - lget(l);
    const int4 r = R[i];
    atomicAdd(&csum[id * 5 + 0], r.x);
    atomicAdd(&csum[id * 5 + 1], r.y);
    atomicAdd(&csum[id * 5 + 2], r.z);
    atomicAdd(&csum[id * 5 + 3], r.w);
    atomicAdd(&csum[id * 5 + 4], 1);
  }
  __threadfence();
  __syncthreads();
  int4* crect = cls_rect + (int64_t)blockIdx.x * cap;
  for (int c = threadIdx.x; c < ncls; c += HC_THREADS) {
    const float s = 1.f / (float)ld_agent(&csum[c * 5 + 4]);
    int* cr = reinterpret_cast<int*>(&crect[c]);
    for (int k = 0; k < 4; k++)
      __hip_atomic_store(&cr[k], hround((float)ld_agent(&csum[c * 5 + k]) * s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __threadfence();
  __syncthreads();
  auto class_rect = [&](int c) {
    const int* cr = reinterpret_cast<const int*>(&crect[c]);
    return make_int4(ld_agent(&cr[0]), ld_agent(&cr[1]), ld_agent(&cr[2]), ld_agent(&cr[3]));
  };
  // small-inside-large filter, output in class order
  int nout = 0;
  for (int c0 = 0; c0 < ncls; c0 += HC_THREADS) {
    const int c = c0 + threadIdx.x;
    int keep = 0;
    int4 r1 = make_int4(0, 0, 0, 0);
    if (c < ncls) {
      r1 = class_rect(c);
      const int n1 = ld_agent(&csum[c * 5 + 4]);
      if (n1 > min_neighbors) {
        keep = 1;
        for (int j = 0; j < ncls; j++) {
          const int n2 = ld_agent(&csum[j * 5 + 4]);
          if (j == c || n2 <= min_neighbors) continue;
          const int4 r2 = class_rect(j);
          const int dx = hround_d(r2.z * eps), dy = hround_d(r2.w * eps);
          if (r1.x >= r2.x - dx && r1.y >= r2.y - dy && r1.x + r1.z <= r2.x + r2.z + dx &&
              r1.y + r1.w <= r2.y + r2.w + dy && (n2 > max(3, n1) || n1 < 3)) {
            keep = 0;
            break;
          }
        }
      }
    }
    int tot;
    const int at = block_excl_scan(keep, sh, tot) + nout;
    if (keep) {
      if (widen) {  // detectFace (FaceForest.cpp:148-158) + intersect (face_utils.cpp:328-346)
        const int ox = (int)(r1.z * 0.05), oy = (int)(r1.z * 0.15);
        const int x1 = r1.x - ox, y1 = r1.y, w1 = r1.z + ox * 2, h1 = r1.w + oy * 2;
        int4 r;
        r.x = x1 < 0 ? 0 : x1;
        r.y = y1 < 0 ? 0 : y1;
        r.z = (x1 + w1 < f.w ? x1 + w1 : f.w) - r.x;
        r.w = (y1 + h1 < f.h ? y1 + h1 : f.h) - r.y;
        if (r.z <= 0 || r.w <= 0) r = make_int4(0, 0, 0, 0);
        r1 = r;
      }
      out[at] = r1;
    }
    nout += tot;
  }
  if (threadIdx.x == 0) n_boxes[blockIdx.x] = nout;
}

// every frame's boxes packed contiguously in frame order (one workgroup)
__global__ __launch_bounds__(HC_THREADS) void k_haar_pack(int n_frames, int cap, const int4* __restrict__ boxes,
                                                           const int32_t* __restrict__ n_boxes,
                                                           int4* __restrict__ packed, int32_t* __restrict__ owner) {
  __shared__ int sh[HC_THREADS / 64 + 1];
  int base = 0;
  for (int f0 = 0; f0 < n_frames; f0 += HC_THREADS) {
    const int f = f0 + threadIdx.x;
    const int n = f < n_frames ? n_boxes[f] : 0;
    int tot;
    const int at = base + block_excl_scan(n, sh, tot);
    for (int i = 0; i < n; i++) {
      packed[at + i] = boxes[(int64_t)f * cap + i];
      owner[at + i] = f;
    }
    base += tot;
  }
}

}  // namespace

void launch_haar_pack(int n_frames, int cap, const int4* boxes, const int32_t* n_boxes, int4* packed, int32_t* owner,
                      hipStream_t s) {
  k_haar_pack<<<1, HC_THREADS, 0, s>>>(n_frames, cap, boxes, n_boxes, packed, owner);
}

void launch_haar_gray(const HaarFrame* frames, int n_frames, int max_pixels, const uint8_t* images, uint8_t* gray,
                      hipStream_t s) {
  const int blocks = std::min(1024, (max_pixels + 255) / 256);
  k_haar_gray<<<dim3(blocks, n_frames), 256, 0, s>>>(frames, images, gray);
}

void launch_haar_pyramid(const HaarLevel* levels, int n_levels, int max_pixels, int max_rows, int max_cols,
                         const uint8_t* gray, uint8_t* scaled, int32_t* sum, uint32_t* sq, hipStream_t s) {
  k_haar_resize<<<dim3(std::min(512, (max_pixels + 256 * HZ_ROWS - 1) / (256 * HZ_ROWS) + 1), n_levels), 256, 0, s>>>(levels, gray,
                                                                                                         scaled);
  k_haar_rows<<<dim3(std::min(256, (max_rows + 1 + 3) / 4), n_levels), 256, 0, s>>>(levels, scaled, sum, sq);
  k_haar_cols<<<dim3((max_cols + 255) / 256, n_levels), 256, 0, s>>>(levels, sum, sq);
}

int haar_cascade_lds(int max_ystep, int ww, int wh) {
  return haar_win_cols(max_ystep, ww) * haar_win_rows(max_ystep, wh) * 4;
}

void launch_haar_cascade(const HaarLevel* levels, int n_levels, int total_tiles, const int32_t* sum, const uint32_t* sq,
                         const HaarWeak* weak, int n_weak, const HaarStage* stages, int n_stages, int ww, int wh,
                         int order_free, int8_t* result, int lds_bytes, hipStream_t s) {
  if (total_tiles <= 0 || n_levels <= 0) return;
  k_haar_cascade<<<total_tiles, HT_THREADS, lds_bytes, s>>>(levels, n_levels, sum, sq, weak, n_weak, stages, n_stages, ww,
                                                            wh, order_free, result);
}

// The grouping of a frame with more raw detections than a workgroup's LDS holds (the overflow re-run, one frame):
// the same connected components of SimilarRects (every label the smallest index of its component), with the
// O(N^2) pair tests spread over the whole chip.  A round: every candidate i takes the smallest label among the
// candidates similar to it (tiles of candidates and their labels staged in LDS; labels only decrease, so reading
// one that another workgroup is lowering at the same time only speeds convergence), then pointer jumping; the
// host repeats rounds until one changes nothing.
constexpr int HL_THREADS = 256;
__global__ __launch_bounds__(HL_THREADS) void k_haar_label_init(const int32_t* __restrict__ n_cand, int cap,
                                                              int* __restrict__ label) {
  const int N = min(n_cand[0], cap);
  for (int i = blockIdx.x * HL_THREADS + threadIdx.x; i < N; i += gridDim.x * HL_THREADS) label[i] = i;
}
__global__ __launch_bounds__(HL_THREADS) void k_haar_label_round(const int4* __restrict__ R, const int32_t* __restrict__ n_cand,
                                                               int cap, int* __restrict__ label, int* __restrict__ changed) {
  __shared__ int4 tr[HL_THREADS];
  __shared__ int tl[HL_THREADS];
  const int N = min(n_cand[0], cap);
  const int i = blockIdx.x * HL_THREADS + threadIdx.x;
  if (blockIdx.x * HL_THREADS >= N) return;  // (whole workgroup: the barriers below stay uniform)
  const int4 ri = i < N ? R[i] : make_int4(0, 0, 0, 0);
  int m = i < N ? __hip_atomic_load(&label[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
  const int m0 = m;
  for (int j0 = 0; j0 < N; j0 += HL_THREADS) {
    const int j = j0 + threadIdx.x;
    if (j < N) {
      tr[threadIdx.x] = R[j];
      tl[threadIdx.x] = __hip_atomic_load(&label[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (i < N) {
      const int n = min(HL_THREADS, N - j0);
      for (int k = 0; k < n; k++)
        if (j0 + k != i && tl[k] < m && similar_rects(ri, tr[k], 0.2)) m = tl[k];
    }
    __syncthreads();
  }
  if (i < N && m < m0) {
    __hip_atomic_fetch_min(&label[i], m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(changed, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
__global__ __launch_bounds__(HL_THREADS) void k_haar_label_jump(const int32_t* __restrict__ n_cand, int cap,
                                                              int* __restrict__ label) {
  const int N = min(n_cand[0], cap);
  for (int i = blockIdx.x * HL_THREADS + threadIdx.x; i < N; i += gridDim.x * HL_THREADS) {
    int l = __hip_atomic_load(&label[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
      const int n = __hip_atomic_load(&label[l], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (n == l) break;
      l = n;
    }
    __hip_atomic_fetch_min(&label[i], l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

int launch_haar_group(const HaarFrame* frames, int n_frames, int max_frame_rows, int32_t* rowcnt,
                       const HaarLevel* levels, const int8_t* result, int cap, int4* cand, int32_t* n_cand,
                       int min_neighbors, int widen, int4* cls_rect, int* cls_sum, int4* boxes, int32_t* n_boxes,
                       int* label_g, hipStream_t s) {
#if FFD_HAAR_COLLECT_SERIAL
  (void)max_frame_rows;
  (void)rowcnt;
  k_haar_collect<<<n_frames, HC_THREADS, 0, s>>>(frames, levels, result, cap, cand, n_cand);
#else
  const int rb = std::max(1, (max_frame_rows + HR_THREADS - 1) / HR_THREADS);
  const int rb_count = (max_frame_rows + HR_THREADS / 64 - 1) / (HR_THREADS / 64);  // (k_haar_rowcount: a wave per row)
  if (max_frame_rows > 0) k_haar_rowcount<<<dim3(n_frames, rb_count), HR_THREADS, 0, s>>>(frames, levels, result, max_frame_rows, rowcnt);
  k_haar_emit<<<dim3(n_frames, rb), HR_THREADS, 0, s>>>(frames, levels, result, max_frame_rows, rowcnt, cap, cand, n_cand);
#endif
  if (cap > HAAR_MAX_CAND) {  // (one frame: the overflow re-run)
    if (min_neighbors > 0) {
      int* changed = label_g + cap;  // (the label buffer holds cap + 1 ints)
      const int grid = (cap + HL_THREADS - 1) / HL_THREADS;
      k_haar_label_init<<<std::min(grid, 1024), HL_THREADS, 0, s>>>(n_cand, cap, label_g);
      // min-label rounds until no label changes: at most cap rounds (a label only decreases); a failed HIP call or
      // running past that bound is reported, never taken as convergence (unconverged labels would group wrongly)
      for (int round = 0;; round++) {
        if (round > cap) return HAAR_GROUP_NO_CONVERGENCE;
        int h = 0;
        if (hipMemsetAsync(changed, 0, sizeof(int), s) != hipSuccess) return HAAR_GROUP_HIP_ERROR;
        k_haar_label_round<<<grid, HL_THREADS, 0, s>>>(cand, n_cand, cap, label_g, changed);
        k_haar_label_jump<<<std::min(grid, 1024), HL_THREADS, 0, s>>>(n_cand, cap, label_g);
        if (hipGetLastError() != hipSuccess || hipMemcpyAsync(&h, changed, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
          return HAAR_GROUP_HIP_ERROR;
        if (!h) break;
      }
    }
    k_haar_group<true><<<n_frames, HC_THREADS, 0, s>>>(frames, cap, cand, n_cand, min_neighbors, widen, cls_rect, cls_sum,
                                                     boxes, n_boxes, label_g);
  }
  else
    k_haar_group<false><<<n_frames, HC_THREADS, 0, s>>>(frames, cap, cand, n_cand, min_neighbors, widen, cls_rect,
                                                      cls_sum, boxes, n_boxes, nullptr);
  return HAAR_GROUP_OK;
}

}  // namespace ffd
