// ffd_train.hip — gfx950 kernels of facial-feature (MPSample) tree training, SURVEY.md §8(f) #3.
//
// Compiled with -ffp-contract=off: every float / double expression rounds as written, so the results
// are bit-identical to the CPU restatement oracle/ffd_train_oracle.cpp (which cites the reference
// lines each step follows).  Host orchestration: ffd_train.cpp.
//
//   channels of a training ROI (ImageSample(img, {0,1,2}, false), ImageSample.cpp:11-20 +
//   FeatureChannelFactory.hpp:35-183), any width:        k_tr_gray_sobel, k_tr_gabor_v, k_tr_gabor_h,
//                                                        k_tr_gabor7, k_tr_quantise, k_tr_integral
//   SplitGen::generateMT's per-stripe mt19937 (SplitGen.hpp:78):            k_tr_mt
//   generateSplit + evalTest + sort + findThreshold + evalSplit per (node, stripe)
//   (SplitGen.hpp:74-101,170-231; MPSample.cpp:86-144,276-297):             k_tr_items
//   findOptimalSplit's first strict maximum over stripes (Tree.hpp:261-289): k_tr_select
//   applyOptimalSplit (Tree.hpp:291-308, SplitGen.hpp:103-167):             k_tr_partition
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "../../include/ffd_numerics.h"
#include "ffd_train.hpp"

namespace ffd_train {

__device__ __forceinline__ int reflect101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) {
    if (i < 0) i = -i;
    if (i >= n) i = 2 * n - 2 - i;
  }
  return i;
}
__device__ __forceinline__ int sat_u8(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }
__device__ __forceinline__ int cv_round(float v) {  // cvRound: half to even; NaN / out of range -> INT_MIN
  if (!(v >= -2147483648.0f && v < 2147483648.0f)) return (int)0x80000000;
  return (int)__builtin_rintf(v);
}

// ------------------------------------------------------------ channels ----
// Scratch layout per image of a channel batch (TrImage offsets): u8 planes [38][h][w] (0 gray,
// 1..35 Gabor, 36 Sobel d/dy, 37 Sobel d/dx), magnitudes f32 [35][h][w], V planes f32 [4][9][h][w]
// (scales 1..4: Vg, then (Vc_q, Vs_q) for q = 1..4), integral planes u32 [38][h+1][w+1].

// gray (channel 0) and Sobel 3x3 with BORDER_REFLECT_101, saturated to u8 (FeatureChannelFactory.hpp:120-141)
__global__ void k_tr_gray_sobel(const TrImage* __restrict__ imgs, const uint8_t* __restrict__ gray, uint8_t* __restrict__ u8) {
  const TrImage im = imgs[blockIdx.y];
  const int w = im.w, h = im.h, n = w * h;
  const uint8_t* g = gray + im.gray_off;
  uint8_t* o = u8 + im.u8_off;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int y = i / w, x = i - y * w;
    auto I = [&](int yy, int xx) { return (int)g[reflect101(yy, h) * w + reflect101(xx, w)]; };
    o[i] = g[i];
    const int dy = (I(y + 1, x - 1) + 2 * I(y + 1, x) + I(y + 1, x + 1)) - (I(y - 1, x - 1) + 2 * I(y - 1, x) + I(y - 1, x + 1));
    const int dx = (I(y - 1, x + 1) + 2 * I(y, x + 1) + I(y + 1, x + 1)) - (I(y - 1, x - 1) + 2 * I(y, x - 1) + I(y + 1, x - 1));
    o[(size_t)36 * n + i] = (uint8_t)sat_u8(dy);
    o[(size_t)37 * n + i] = (uint8_t)sat_u8(dx);
  }
}

// Gabor scales 1..4, vertical pass of the separable definition (include/ffd_gabor.h; the operation
// order of oracle/ffd_oracle.cpp gabor_sep_mag): per pixel Vg and (Vc_q, Vs_q), q = 1..4.
__global__ void k_tr_gabor_v(const TrImage* __restrict__ imgs, const uint8_t* __restrict__ gray,
                             const ffd_gabor_sep* __restrict__ sep, float* __restrict__ vbuf) {
  const TrImage im = imgs[blockIdx.y];
  const int nu = 1 + blockIdx.z, w = im.w, h = im.h, n = w * h;
  const ffd_gabor_sep& s = sep[nu];
  const int R = s.R;
  const uint8_t* g = gray + im.gray_off;
  float* V = vbuf + im.v_off + (size_t)(nu - 1) * 9 * n;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int y = i / w, x = i - y * w;
    auto P = [&](int yy) { return (float)g[reflect101(yy, h) * w + x]; };
    float vg = 0.f, c[4] = {0.f, 0.f, 0.f, 0.f}, sv[4] = {0.f, 0.f, 0.f, 0.f};
    for (int t = R; t >= 1; t--) {
      const float a = P(y + t), b = P(y - t), S = a + b, D = a - b;
      vg = __builtin_fmaf(s.g[t], S, vg);
#pragma unroll
      for (int q = 0; q < 4; q++) {
        c[q] = __builtin_fmaf(s.vc[q][t], S, c[q]);
        sv[q] = __builtin_fmaf(s.vs[q][t], D, sv[q]);
      }
    }
    const float p0 = P(y);
    vg = __builtin_fmaf(s.g[0], p0, vg);
    V[i] = vg;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      V[(size_t)(1 + 2 * q) * n + i] = __builtin_fmaf(s.vc[q][0], p0, c[q]);
      V[(size_t)(2 + 2 * q) * n + i] = __builtin_fmaf(s.vs[q][0], p0, sv[q]);
    }
  }
}

// Gabor scales 1..4, horizontal pass + magnitude (gabor_sep_mag's H loop); blockIdx.z = index - 7.
__global__ void k_tr_gabor_h(const TrImage* __restrict__ imgs, const ffd_gabor_sep* __restrict__ sep,
                             const float* __restrict__ vbuf, float* __restrict__ mag) {
  const TrImage im = imgs[blockIdx.y];
  const int index = 7 + blockIdx.z, nu = index / 7, mu = index % 7, w = im.w, h = im.h, n = w * h;
  const ffd_gabor_sep& s = sep[nu];
  constexpr int GP[7] = {0, 1, 2, 3, 4, 3, 2}, GQ[7] = {0, 1, 2, 3, 4, 3, 2};  // FFD_GABOR_P / _Q / _SGN
  const int R = s.R, p = GP[mu], q = GQ[mu];
  const float sgn = mu >= 5 ? -1.f : 1.f;
  const float* V = vbuf + im.v_off + (size_t)(nu - 1) * 9 * n;
  const float* Vg = V;
  const float* Vc = V + (size_t)(q > 0 ? 2 * q - 1 : 0) * n;
  const float* Vs = V + (size_t)(q > 0 ? 2 * q : 0) * n;
  float* M = mag + im.mag_off + (size_t)index * n;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int y = i / w, x = i - y * w;
    float re = 0.f, imv = 0.f, dc = 0.f, A = 0.f, B = 0.f, C = 0.f, E = 0.f;
    for (int t = -R; t <= R; t++) {
      const int j = y * w + reflect101(x + t, w);
      const int at = t < 0 ? -t : t;
      const float gv = Vg[j];
      dc = __builtin_fmaf(s.g[at], gv, dc);
      if (mu == 0) {
        const float hs = t < 0 ? -s.hs[0][at] : s.hs[0][at];
        re = __builtin_fmaf(s.hc[0][at], gv, re);
        imv = __builtin_fmaf(hs, gv, imv);
      } else if (mu == 4) {
        re = __builtin_fmaf(s.g[at], Vc[j], re);
        imv = __builtin_fmaf(s.g[at], Vs[j], imv);
      } else {
        const float hc = s.hc[p][at], hs = t < 0 ? -s.hs[p][at] : s.hs[p][at];
        A = __builtin_fmaf(hc, Vc[j], A);
        C = __builtin_fmaf(hc, Vs[j], C);
        B = __builtin_fmaf(hs, Vs[j], B);
        E = __builtin_fmaf(hs, Vc[j], E);
      }
    }
    if (mu != 0 && mu != 4) {
      re = sgn > 0 ? A - B : A + B;
      imv = sgn > 0 ? C + E : C - E;
    }
    re = __builtin_fmaf(-s.c, dc, re);
    const float r2 = re * re, i2 = imv * imv;
    M[i] = __builtin_sqrtf(i2 + r2);
  }
}

// Gabor 7x7 (scale 0): OpenCV's direct Filter2D order (row-major taps, s = s + k * p, no FMA);
// taps: [mu][49] re then [mu][49] im.  blockIdx.z = mu.
__global__ void k_tr_gabor7(const TrImage* __restrict__ imgs, const uint8_t* __restrict__ gray,
                            const float* __restrict__ taps, float* __restrict__ mag) {
  const TrImage im = imgs[blockIdx.y];
  const int mu = blockIdx.z, w = im.w, h = im.h, n = w * h;
  const uint8_t* g = gray + im.gray_off;
  const float* kr = taps + mu * 98;
  const float* ki = kr + 49;
  float* M = mag + im.mag_off + (size_t)mu * n;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int y = i / w, x = i - y * w;
    float re = 0.f, imv = 0.f;
    for (int r = 0; r < 7; r++) {
      const uint8_t* row = g + reflect101(y + r - 3, h) * w;
      for (int c = 0; c < 7; c++) {
        const float pv = (float)row[reflect101(x + c - 3, w)];
        re = re + kr[r * 7 + c] * pv;
        imv = imv + ki[r * 7 + c] * pv;
      }
    }
    const float r2 = re * re, i2 = imv * imv;
    M[i] = __builtin_sqrtf(i2 + r2);
  }
}

// normalize(NORM_MINMAX, 0, 1) + convertTo(CV_8U, 255) of one magnitude plane (FeatureChannelFactory.hpp:271-286);
// one 256-thread workgroup per (image, Gabor index): blockIdx.x = index, blockIdx.y = image.
__global__ __launch_bounds__(256) void k_tr_quantise(const TrImage* __restrict__ imgs, const float* __restrict__ mag,
                                                    uint8_t* __restrict__ u8) {
  const TrImage im = imgs[blockIdx.y];
  const int idx = blockIdx.x, n = im.w * im.h;
  const float* M = mag + im.mag_off + (size_t)idx * n;
  uint8_t* o = u8 + im.u8_off + (size_t)(1 + idx) * n;
  float mn = M[0], mx = M[0];
  for (int i = threadIdx.x; i < n; i += 256) { mn = fminf(mn, M[i]); mx = fmaxf(mx, M[i]); }
  __shared__ float smn[256], smx[256];
  __shared__ float s_sf, s_hf;
  smn[threadIdx.x] = mn;
  smx[threadIdx.x] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int t = 1; t < 256; t++) { mn = fminf(mn, smn[t]); mx = fmaxf(mx, smx[t]); }
    const double smin = mn, smax = mx, dmin = 0, dmax = 1;
    const double scale = (dmax - dmin) * (smax - smin > 2.220446049250313e-16 ? 1. / (smax - smin) : 0);
    const double shift = dmin - smin * scale;
    s_sf = (float)scale;
    s_hf = (float)shift;
  }
  __syncthreads();
  const float sf = s_sf, hf = s_hf;
  for (int i = threadIdx.x; i < n; i += 256) {
    const float v = M[i] * sf + hf;
    o[i] = (uint8_t)sat_u8(cv_round(v * 255.f + 0.f));
  }
}

// cv::integral of one u8 plane into u32 (h+1) x (w+1), exact: rows then columns.
// blockIdx.x = channel, blockIdx.y = image.
__global__ __launch_bounds__(256) void k_tr_integral(const TrImage* __restrict__ imgs, const uint8_t* __restrict__ u8,
                                                    uint32_t* __restrict__ chan) {
  const TrImage im = imgs[blockIdx.y];
  const int c = blockIdx.x, w = im.w, h = im.h, W1 = w + 1;
  const uint8_t* src = u8 + im.u8_off + (size_t)c * w * h;
  uint32_t* I = chan + im.ch_off + (size_t)c * W1 * (h + 1);
  for (int x = threadIdx.x; x <= w; x += 256) I[x] = 0;
  for (int y = threadIdx.x; y < h; y += 256) {
    uint32_t* r = I + (size_t)(y + 1) * W1;
    uint32_t s = 0;
    r[0] = 0;
    for (int x = 0; x < w; x++) { s += src[y * w + x]; r[x + 1] = s; }
  }
  __syncthreads();
  for (int x = 1 + threadIdx.x; x <= w; x += 256) {
    uint32_t s = 0;
    for (int y = 1; y <= h; y++) { s += I[(size_t)y * W1 + x]; I[(size_t)y * W1 + x] = s; }
  }
}

// ------------------------------------------------------------ training ----
// mt19937 (== boost::mt19937) seeded with `seed`: its first MT_WIN outputs.  Output i < 227 of the
// first twist only needs the initial state x[i], x[i + 1], x[i + 397], so one lane walks the seeding
// recurrence once, keeping x[0..MT_WIN] in registers, and tempers output i when x[397 + i] appears.
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

// The first MT_WIN outputs of mt19937(seed) into o[] (one thread).
__device__ __forceinline__ void mt_first(uint32_t seed, uint32_t* __restrict__ o) {
  uint32_t x[MT_WIN + 1];
  uint32_t cur = seed;
  x[0] = cur;
#pragma unroll
  for (int j = 1; j <= MT_WIN; j++) {
    cur = 1812433253u * (cur ^ (cur >> 30)) + (uint32_t)j;
    x[j] = cur;
  }
#pragma unroll 4
  for (int j = MT_WIN + 1; j < 397; j++) cur = 1812433253u * (cur ^ (cur >> 30)) + (uint32_t)j;
#pragma unroll
  for (int i = 0; i < MT_WIN; i++) {
    cur = 1812433253u * (cur ^ (cur >> 30)) + (uint32_t)(397 + i);
    const uint32_t y = (x[i] & 0x80000000u) | (x[i + 1] & 0x7fffffffu);
    o[i] = mt_temper(cur ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u));
  }
}

// one thread per item (node, stripe): the stripe generator of SplitGen::generateMT, seeded with
// (stripe + 1) * (split_seed + heap index of the node) (oracle/ffd_train_oracle.cpp: time(NULL)'s stand-in)
__global__ __launch_bounds__(256) void k_tr_mt(const TrNode* __restrict__ nodes, int n_items, int ntests,
                                              uint32_t split_seed, uint32_t* __restrict__ raw) {
  const int item = blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= n_items) return;
  const int node = item / ntests, stripe = item - node * ntests;
  mt_first((uint32_t)((uint64_t)(stripe + 1) * (uint64_t)(split_seed + nodes[node].heap)), raw + (size_t)item * MT_WIN);
}

// Boost.Random generate_uniform_int over a window of engine outputs (wave-uniform): bucket division
// with rejection; flags the item when the window runs out (never met: a rejection has probability
// below 2^-22 per draw, the window leaves 14 spare outputs).
struct Draws {
  const uint32_t* raw;
  int cur;
  bool bad;
  __device__ int operator()(int lo, int hi) {
    const uint32_t range = (uint32_t)(hi - lo);
    if (range == 0) return lo;
    uint32_t bucket = 0xFFFFFFFFu / (range + 1u);
    if (0xFFFFFFFFu % (range + 1u) == range) ++bucket;
    for (;;) {
      if (cur >= MT_WIN) { bad = true; return lo; }
      const uint32_t r = raw[cur++] / bucket;
      if (r <= range) return lo + (int)r;
    }
  }
};

// SimplePatchFeature::generate(patch_size, rng, 38) (ImageSample.hpp:35-81); smax = (int)((ps - 1) * 0.75)
__device__ __forceinline__ TrFeature gen_feature(Draws& d, int ps, int smax) {
  TrFeature f;
  f.ch = d(0, NCH - 1);
  f.r[2] = d(1, smax);
  f.r[3] = d(1, smax);
  f.r[6] = d(1, smax);
  f.r[7] = d(1, smax);
  f.r[0] = d(0, ps - f.r[2] - 1);
  f.r[1] = d(0, ps - f.r[3] - 1);
  f.r[4] = d(0, ps - f.r[6] - 1);
  f.r[5] = d(0, ps - f.r[7] - 1);
  return f;
}

// ImageSample::evalTest, non-integral branch (ImageSample.cpp:40-47): rectangle sums from the exact
// integral planes, (int)(sum / (float)area) = floor(sum / area) (for sum < 2^24 the float quotient
// never rounds up to the next integer: the gap k - sum / area >= 1 / area > k 2^-24).  Computed as
// (int)fma(sum, rcp(area), 0.00075) for area <= 484, i.e. patch sizes up to 31 (equal for every sum in
// [0, 255 area]: tests/test_numerics.py), and as the integer quotient above that (patch sizes up to 64
// give areas up to 47 x 47; the rectangle is wave-uniform, so the branch does not diverge).
__device__ __forceinline__ int eval_sample(const TrImage* __restrict__ imgs, const TrSample& s, const TrFeature& f,
                                           const uint32_t* __restrict__ chan) {
  const TrImage im = imgs[s.img];
  const int W1 = im.w + 1;
  const uint32_t* I = chan + im.ch_off + (size_t)f.ch * W1 * (im.h + 1);
  auto mean = [&](int rx, int ry, int rw, int rh) {
    const uint32_t* p = I + (size_t)(s.y + ry) * W1 + (s.x + rx);
    const uint32_t S = p[(size_t)rh * W1 + rw] - p[rw] - p[(size_t)rh * W1] + p[0];
    const uint32_t area = (uint32_t)(rw * rh);
    if (area > 484u) return (int)(S / area);
    return (int)__builtin_fmaf((float)S, __builtin_amdgcn_rcpf((float)area), 0.00075f);
  };
  return mean(f.r[0], f.r[1], f.r[2], f.r[3]) - mean(f.r[4], f.r[5], f.r[6], f.r[7]);
}

__device__ __forceinline__ uint64_t lanes_below() {
  const int l = __lane_id();
  return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// Stable counting sort of a node's samples by feature value (std::sort of (value, index) pairs):
// ctr[v + 255] starts at the number of values below v; the samples are ranked within each 64-sample
// chunk by a 9-ballot match on the value and scattered to out[ctr + rank]; the highest lane of each
// value group then advances the counter.  Every lane of the wave calls this (uniform control flow).
__device__ __forceinline__ void scatter_sorted(const TrImage* __restrict__ imgs, const TrSample* __restrict__ samples,
                                               const int32_t* __restrict__ list, int n, const TrFeature& f,
                                               const uint32_t* __restrict__ chan, int* __restrict__ ctr,
                                               int32_t* __restrict__ out) {
  const int lane = __lane_id();
  for (int c0 = 0; c0 < n; c0 += 64) {
    const int i = c0 + lane;
    const bool act = i < n;
    int gid = 0, key = 0;
    if (act) {
      gid = list[i];
      key = eval_sample(imgs, samples[gid], f, chan) + 255;
    }
    uint64_t m = __ballot(act);
#pragma unroll
    for (int b = 0; b < 9; b++) {
      const bool bit = (key >> b) & 1;
      const uint64_t bb = __ballot(bit);
      m &= bit ? bb : ~bb;
    }
    int base = 0;
    if (act) base = ctr[key];
    __builtin_amdgcn_wave_barrier();
    if (act) {
      out[base + __popcll(m & lanes_below())] = gid;
      if ((m >> lane) == 1ull) ctr[key] = base + __popcll(m);  // the group's highest lane
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// Per-wave LDS of k_tr_items
struct ItemLds {
  int hist[512];   // counts, then the exclusive prefix (values below v), then the scatter counters
  int ku[TR_THR + 1];        // unique valid split points (ascending)
  int tj[TR_THR], kj[TR_THR], jm[TR_THR];
  int nu;
  float sA[TR_THR][10], sB[TR_THR][10];
  double info[TR_THR];
};

__device__ __forceinline__ double entropy_parts(const float* sum, int cnt) {  // MPSample.cpp:276-297
  const float sf = (float)(1.0 / (double)(float)cnt);
  double e = 0;
#pragma unroll
  for (int p = 0; p < 10; p++) {
    const float pb = sum[p] * sf + 0.0f;
    if (pb > 0) e += (double)pb * ffd_log((double)pb);
  }
  return e;
}

// One wave per item = (node, stripe): the stripe's feature, every sample's value, min / max and
// histogram, the 25 thresholds, the stable sort, the float sums of the part probabilities over both
// sides of every threshold (sequential in sorted order, as the reference adds them), the information
// gains, and the stripe's best threshold (first strict maximum).
__global__ __launch_bounds__(256) void k_tr_items(TrItemsArgs A) {
  __shared__ ItemLds L[4];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int item = blockIdx.x * 4 + wv;
  if (item >= A.n_items) return;  // whole waves only: no workgroup barrier below
  ItemLds& S = L[wv];
  const int node = item / A.ntests;
  const TrNode nd = A.nodes[node];
  const int n = nd.cnt;
  const int32_t* list = A.list + nd.beg;
  Draws d{A.raw + (size_t)item * MT_WIN, 0, false};
  const TrFeature f = gen_feature(d, A.ps, A.smax);
  // pass 1: values -> histogram, min / max
  for (int b = lane; b < 512; b += 64) S.hist[b] = 0;
  __builtin_amdgcn_wave_barrier();
  int vmin = 1 << 20, vmax = -(1 << 20);
  for (int i = lane; i < n; i += 64) {
    const int v = eval_sample(A.imgs, A.samples[list[i]], f, A.chan);
    vmin = min(vmin, v);
    vmax = max(vmax, v);
    atomicAdd(&S.hist[v + 255], 1);
  }
#pragma unroll
  for (int sh = 32; sh >= 1; sh >>= 1) {
    vmin = min(vmin, __shfl_xor(vmin, sh));
    vmax = max(vmax, __shfl_xor(vmax, sh));
  }
  __builtin_amdgcn_wave_barrier();
  // exclusive prefix of the histogram (8 bins per lane)
  {
    int loc[8], run = 0;
#pragma unroll
    for (int u = 0; u < 8; u++) { loc[u] = S.hist[lane * 8 + u]; run += loc[u]; }
    int incl = run;
#pragma unroll
    for (int sh = 1; sh < 64; sh <<= 1) {
      const int t = __shfl_up(incl, sh);
      if (lane >= sh) incl += t;
    }
    int ex = incl - run;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int u = 0; u < 8; u++) { S.hist[lane * 8 + u] = ex; ex += loc[u]; }
  }
  __builtin_amdgcn_wave_barrier();
  // thresholds (findThreshold, SplitGen.hpp:170-231): uniform in [0, range] + min, wave-uniform
  const int range = vmax - vmin;
  int nvalid = 0;
  if (range > 0) {
    for (int j = 0; j < A.nthr; j++) {
      const int t = d(0, range) + vmin;
      const int k = S.hist[t + 255];  // lower_bound: values below t
      if (lane == 0) { S.tj[j] = t; S.kj[j] = (k < 2 || n - k < 2) ? -1 : k; }
      nvalid += (k < 2 || n - k < 2) ? 0 : 1;
    }
  }
  if (d.bad && lane == 0) atomicOr(A.error, 1);
  if (nvalid == 0) {
    if (lane == 0) { A.out_info[item] = -1.7976931348623157e308; A.out_thr[item] = 0; A.out_k[item] = 0; }
    return;
  }
  __builtin_amdgcn_wave_barrier();
  // unique split points, ascending; jm[j] = slot of threshold j
  if (lane == 0) {
    int m = 0;
    for (int j = 0; j < A.nthr; j++) {
      const int k = S.kj[j];
      if (k < 0) continue;
      int pos = 0;
      while (pos < m && S.ku[pos] < k) pos++;
      if (pos < m && S.ku[pos] == k) continue;
      for (int q = m; q > pos; q--) S.ku[q] = S.ku[q - 1];
      S.ku[pos] = k;
      m++;
    }
    S.nu = m;
    S.ku[m] = 1 << 30;
    for (int j = 0; j < A.nthr; j++) {
      const int k = S.kj[j];
      int pos = 0;
      if (k >= 0) while (S.ku[pos] != k) pos++;
      S.jm[j] = k < 0 ? -1 : pos;
    }
  }
  __builtin_amdgcn_wave_barrier();
  // pass 2: stable sort (the scatter counters start at the prefix)
  int32_t* sorted = A.sorted + nd.sorted_off + (size_t)(item - node * A.ntests) * n;
  scatter_sorted(A.imgs, A.samples, list, n, f, A.chan, S.hist, sorted);
  __threadfence();  // the other lanes' scattered entries are read below
  __builtin_amdgcn_wave_barrier();
  // pass 3: sequential float sums in sorted order.  Pair q = lane + 64u -> chain c = q / 10, part
  // p = q % 10; chain 0 runs [0, n) and records its prefix at each unique split point; chain 1 + m
  // runs [ku[m], n).
  const int nu = S.nu;
  int start[5], end[5], part[5], chain[5];
  float acc[5];
#pragma unroll
  for (int u = 0; u < 5; u++) {
    const int q = lane + 64 * u, c = q / 10;
    part[u] = q - c * 10;
    chain[u] = c;
    acc[u] = 0.f;
    start[u] = 0;
    end[u] = 0;
    if (q < 260 && c <= nu) {
      start[u] = c == 0 ? 0 : S.ku[c - 1];
      end[u] = n;
    }
  }
  int rec = 0;  // chain 0: next split point to record
  const float* prob = A.prob;
  for (int s = 0; s < n; s++) {
#pragma unroll
    for (int u = 0; u < 5; u++) {
      const int pos = start[u] + s;
      if (pos < end[u]) acc[u] += prob[(size_t)sorted[pos] * 10 + part[u]];
    }
    if (lane < 10 && s + 1 == S.ku[rec]) {  // u = 0, chain 0
      S.sA[rec][lane] = acc[0];
      rec++;
    }
  }
#pragma unroll
  for (int u = 0; u < 5; u++)
    if (end[u] > 0 && chain[u] >= 1) S.sB[chain[u] - 1][part[u]] = acc[u];
  __builtin_amdgcn_wave_barrier();
  // evalSplit per threshold (MPSample.cpp:103-144, mode 1)
  if (lane < A.nthr) {
    const int m = S.jm[lane];
    double info = -1.7976931348623157e308;
    if (m >= 0) {
      const int k = S.ku[m];
      const double ea = entropy_parts(S.sA[m], k), eb = entropy_parts(S.sB[m], n - k);
      info = (ea * (double)k + eb * (double)(n - k)) / (double)n;
    }
    S.info[lane] = info;
  }
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) {
    double best = -1.7976931348623157e308;
    int bt = 0, bk = 0;
    for (int j = 0; j < A.nthr; j++)
      if (S.jm[j] >= 0 && S.info[j] > best) { best = S.info[j]; bt = S.tj[j]; bk = S.ku[S.jm[j]]; }
    A.out_info[item] = best;
    A.out_thr[item] = bt;
    A.out_k[item] = bk;
  }
}

// findOptimalSplit (Tree.hpp:261-289): the first stripe with the strictly largest info; -1 if none
// beats the initial lowest().  One workgroup per node.
__global__ __launch_bounds__(256) void k_tr_select(int ntests, const double* __restrict__ info, const int* __restrict__ thr,
                                                  const int* __restrict__ kk, TrBest* __restrict__ best) {
  const int node = blockIdx.x;
  const double* I = info + (size_t)node * ntests;
  double b = -1.7976931348623157e308;
  int bs = -1;
  for (int s = threadIdx.x; s < ntests; s += 256)
    if (I[s] > b) { b = I[s]; bs = s; }
  __shared__ double sb[256];
  __shared__ int ss[256];
  sb[threadIdx.x] = b;
  ss[threadIdx.x] = bs;
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if (threadIdx.x < w) {
      const double o = sb[threadIdx.x + w];
      const int os = ss[threadIdx.x + w];
      if (os >= 0 && (ss[threadIdx.x] < 0 || o > sb[threadIdx.x] || (o == sb[threadIdx.x] && os < ss[threadIdx.x]))) {
        sb[threadIdx.x] = o;
        ss[threadIdx.x] = os;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    TrBest r;
    r.stripe = ss[0];
    r.info = sb[0];
    r.thr = ss[0] >= 0 ? thr[(size_t)node * ntests + ss[0]] : 0;
    r.k = ss[0] >= 0 ? kk[(size_t)node * ntests + ss[0]] : 0;
    best[node] = r;
  }
}

// applyOptimalSplit (Tree.hpp:291-308): the node's samples sorted by the chosen feature's value into
// the next level's list; the children are its two slices at the split point.  One wave per node.
__global__ __launch_bounds__(64) void k_tr_partition(const TrNode* __restrict__ nodes, const TrFeature* __restrict__ feats,
                                                    const TrImage* __restrict__ imgs, const TrSample* __restrict__ samples,
                                                    const uint32_t* __restrict__ chan, const int32_t* __restrict__ list,
                                                    int32_t* __restrict__ next) {
  __shared__ int hist[512];
  const TrNode nd = nodes[blockIdx.x];
  const TrFeature f = feats[blockIdx.x];
  const int lane = threadIdx.x, n = nd.cnt;
  for (int b = lane; b < 512; b += 64) hist[b] = 0;
  __builtin_amdgcn_wave_barrier();
  for (int i = lane; i < n; i += 64) atomicAdd(&hist[eval_sample(imgs, samples[list[nd.beg + i]], f, chan) + 255], 1);
  __builtin_amdgcn_wave_barrier();
  int loc[8], run = 0;
#pragma unroll
  for (int u = 0; u < 8; u++) { loc[u] = hist[lane * 8 + u]; run += loc[u]; }
  int incl = run;
#pragma unroll
  for (int sh = 1; sh < 64; sh <<= 1) {
    const int t = __shfl_up(incl, sh);
    if (lane >= sh) incl += t;
  }
  int ex = incl - run;
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int u = 0; u < 8; u++) { hist[lane * 8 + u] = ex; ex += loc[u]; }
  __builtin_amdgcn_wave_barrier();
  scatter_sorted(imgs, samples, list + nd.beg, n, f, chan, hist, next + nd.beg);
}


// ----------------------------------------------------------- head pose ----
// HeadPoseSample::evalSplit (HeadPoseSample.cpp:64-87) from the class counts of the two sides:
// c[0..4] = positives per label, c[5] = background.  entropie (:120-143) and gain2 (:228-248) sum 1s,
// labels and squared labels in double in the reference: exact integers, equal to the counts' values.
__device__ __forceinline__ double hp_entropie(double p, int size) {
  double e = 0;
  const double p_pos = p / (double)size;
  if (p_pos > 0) e += p_pos * ffd_log(p_pos);
  const double p_neg = ((double)size - p) / (double)size;
  if (p_neg > 0) e += p_neg * ffd_log(p_neg);
  return e;
}
__device__ __forceinline__ double hp_gain2(double n, double sum, double sq_sum) {
  const double mean = sum / n;
  const double variance = (sq_sum / n) - (mean * mean);
  return -variance;
}
__device__ __forceinline__ double hp_eval_split(const int* a, const int* b, int mode) {
  int pa = 0, pb = 0, sa = 0, sb = 0, qa = 0, qb = 0;
#pragma unroll
  for (int l = 0; l < 5; l++) {
    pa += a[l]; pb += b[l];
    sa += l * a[l]; sb += l * b[l];
    qa += l * l * a[l]; qb += l * l * b[l];
  }
  const int na = pa + a[5], nb = pb + b[5];
  if (mode < 50) {
    const double ea = hp_entropie((double)pa, na), eb = hp_entropie((double)pb, nb);
    return (ea * (double)na + eb * (double)nb) / (double)(na + nb);
  }
  const double ga = hp_gain2((double)pa, (double)sa, (double)qa), gb = hp_gain2((double)pb, (double)sb, (double)qb);
  return (ga * (double)pa + gb * (double)pb) / (double)(pb + pa);
}

// One workgroup per stripe of ONE node (the depth-first search order fixes the node's split mode):
// the stripe's feature, every sample's value into a per-class histogram (6 x 512 bins in LDS), its
// exclusive prefix, the 25 thresholds, the class counts below each threshold (lower_bound) and the
// information gains; the stripe's best threshold is the first strict maximum (SplitGen.hpp:170-231).
__global__ __launch_bounds__(256) void k_hp_items(HpItemsArgs A) {
  __shared__ uint32_t raw[MT_WIN];
  __shared__ int hist[6][512];
  __shared__ int s_lo, s_hi;
  __shared__ double s_info[TR_THR];
  __shared__ int s_thr[TR_THR];
  const int stripe = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) {
    mt_first((uint32_t)((uint64_t)(stripe + 1) * (uint64_t)A.T), raw);
    s_lo = 1 << 20;
    s_hi = -(1 << 20);
  }
  for (int b = tid; b < 6 * 512; b += 256) (&hist[0][0])[b] = 0;
  __syncthreads();
  Draws d{raw, 0, false};
  const TrFeature f = gen_feature(d, A.ps, A.smax);
  int vmin = 1 << 20, vmax = -(1 << 20);
  for (int i = tid; i < A.n; i += 256) {
    const int gid = A.list[i];
    const int v = eval_sample(A.imgs, A.samples[gid], f, A.chan);
    vmin = min(vmin, v);
    vmax = max(vmax, v);
    atomicAdd(&hist[A.cls[gid]][v + 255], 1);
  }
#pragma unroll
  for (int sh = 32; sh >= 1; sh >>= 1) {
    vmin = min(vmin, __shfl_xor(vmin, sh));
    vmax = max(vmax, __shfl_xor(vmax, sh));
  }
  if (lane == 0) {
    atomicMin(&s_lo, vmin);
    atomicMax(&s_hi, vmax);
  }
  __syncthreads();
  for (int c = wv; c < 6; c += 4) {  // exclusive prefix per class, 8 bins per lane
    int loc[8], run = 0;
#pragma unroll
    for (int u = 0; u < 8; u++) { loc[u] = hist[c][lane * 8 + u]; run += loc[u]; }
    int incl = run;
#pragma unroll
    for (int sh = 1; sh < 64; sh <<= 1) {
      const int t = __shfl_up(incl, sh);
      if (lane >= sh) incl += t;
    }
    int ex = incl - run;
#pragma unroll
    for (int u = 0; u < 8; u++) { hist[c][lane * 8 + u] = ex; ex += loc[u]; }
  }
  __syncthreads();
  if (wv != 0) return;
  const int lo = s_lo, range = s_hi - lo;
  double info = -1.7976931348623157e308;
  int thr = 0;
  if (range > 0) {
    int my_t = 0;
    for (int j = 0; j < A.nthr; j++) {  // wave-uniform draws
      const int t = d(0, range) + lo;
      if (lane == j) my_t = t;
    }
    if (lane < A.nthr) {
      int a[6], b[6], na = 0;
#pragma unroll
      for (int c = 0; c < 6; c++) {
        a[c] = hist[c][my_t + 255];
        b[c] = hist[c][511] - a[c];  // bin 511 is never filled: its prefix is the class total
        na += a[c];
      }
      const bool ok = na >= 2 && A.n - na >= 2;
      s_info[lane] = ok ? hp_eval_split(a, b, A.mode) : 0.0;
      s_thr[lane] = ok ? my_t : INT_MIN;
    }
    __builtin_amdgcn_wave_barrier();
    if (lane == 0)
      for (int j = 0; j < A.nthr; j++)
        if (s_thr[j] != INT_MIN && s_info[j] > info) { info = s_info[j]; thr = s_thr[j]; }
  }
  if (lane == 0) {
    if (d.bad) atomicOr(A.error, 1);
    A.out_info[stripe] = info;
    A.out_thr[stripe] = thr;
  }
}

// findOptimalSplit + applyOptimalSplit for one node (Tree.hpp:135-166,261-308): the first stripe with the
// strictly largest gain, its feature from the stripe's generator, and the node's samples split at the
// threshold (value < threshold -> left) into out[0, nA) and out[nA, n), with each side's class counts.
// The order inside a side is free: every head-pose quantity is a count.  One workgroup.
__global__ __launch_bounds__(1024) void k_hp_split(HpSplitArgs A) {
  __shared__ double sb[1024];
  __shared__ int ss[1024];
  __shared__ uint32_t raw[MT_WIN];
  __shared__ int cnt[2], hs[2][6];
  const int tid = threadIdx.x, lane = tid & 63;
  double b = -1.7976931348623157e308;
  int bs = -1;
  for (int s = tid; s < A.ntests; s += 1024)
    if (A.info[s] > b) { b = A.info[s]; bs = s; }
  sb[tid] = b;
  ss[tid] = bs;
  if (tid < 2) cnt[tid] = 0;
  if (tid < 12) (&hs[0][0])[tid] = 0;
  __syncthreads();
  for (int w = 512; w >= 1; w >>= 1) {
    if (tid < w) {
      const double o = sb[tid + w];
      const int os = ss[tid + w];
      if (os >= 0 && (ss[tid] < 0 || o > sb[tid] || (o == sb[tid] && os < ss[tid]))) {
        sb[tid] = o;
        ss[tid] = os;
      }
    }
    __syncthreads();
  }
  const int best = ss[0];
  if (best < 0) {
    if (tid == 0) A.res->stripe = -1;
    return;
  }
  if (tid == 0) mt_first((uint32_t)((uint64_t)(best + 1) * (uint64_t)A.T), raw);
  __syncthreads();
  Draws d{raw, 0, false};
  const TrFeature f = gen_feature(d, A.ps, A.smax);
  const int thr = A.thr[best];
  const uint64_t below = lanes_below();
  for (int i0 = tid - lane; i0 < A.n; i0 += 1024) {  // whole waves: uniform trip count for the ballots
    const int i = i0 + lane;
    const bool act = i < A.n;
    int gid = 0, c = 0;
    bool left = false;
    if (act) {
      gid = A.list[i];
      c = A.cls[gid];
      left = eval_sample(A.imgs, A.samples[gid], f, A.chan) < thr;
    }
    const uint64_t mA = __ballot(act && left), mB = __ballot(act && !left);
    int baseA = 0, baseB = 0;
    if (lane == 0) {
      baseA = atomicAdd(&cnt[0], __popcll(mA));
      baseB = atomicAdd(&cnt[1], __popcll(mB));
    }
    baseA = __shfl(baseA, 0);
    baseB = __shfl(baseB, 0);
    if (act) {
      if (left) A.out[baseA + __popcll(mA & below)] = gid;
      else A.out[A.n - 1 - (baseB + __popcll(mB & below))] = gid;
      atomicAdd(&hs[left ? 0 : 1][c], 1);
    }
  }
  __syncthreads();
  if (tid == 0) {
    HpSplitResult r;
    r.info = sb[0];
    r.stripe = best;
    r.thr = thr;
    r.na = cnt[0];
    r.nb = cnt[1];
    r.ch = f.ch;
    for (int j = 0; j < 8; j++) r.rect[j] = f.r[j];
    for (int c = 0; c < 6; c++) { r.ha[c] = hs[0][c]; r.hb[c] = hs[1][c]; }
    r.bad = d.bad ? 1 : 0;
    *A.res = r;
  }
}

// ------------------------------------------------------------ launchers ----
void launch_channels(const TrImage* d_imgs, int n_img, int max_px, const uint8_t* gray, const ffd_gabor_sep* sep,
                     const float* taps7, uint8_t* u8, float* mag, float* vbuf, uint32_t* chan, hipStream_t s) {
  const int bx = (max_px + 255) / 256;
  hipLaunchKernelGGL(k_tr_gray_sobel, dim3(bx, n_img), dim3(256), 0, s, d_imgs, gray, u8);
  hipLaunchKernelGGL(k_tr_gabor_v, dim3(bx, n_img, 4), dim3(256), 0, s, d_imgs, gray, sep, vbuf);
  hipLaunchKernelGGL(k_tr_gabor7, dim3(bx, n_img, 7), dim3(256), 0, s, d_imgs, gray, taps7, mag);
  hipLaunchKernelGGL(k_tr_gabor_h, dim3(bx, n_img, 28), dim3(256), 0, s, d_imgs, sep, vbuf, mag);
  hipLaunchKernelGGL(k_tr_quantise, dim3(35, n_img), dim3(256), 0, s, d_imgs, mag, u8);
  hipLaunchKernelGGL(k_tr_integral, dim3(NCH, n_img), dim3(256), 0, s, d_imgs, u8, chan);
}

void launch_mt(const TrNode* nodes, int n_items, int ntests, uint32_t split_seed, uint32_t* raw, hipStream_t s) {
  hipLaunchKernelGGL(k_tr_mt, dim3((n_items + 255) / 256), dim3(256), 0, s, nodes, n_items, ntests, split_seed, raw);
}

void launch_items(const TrItemsArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_tr_items, dim3((a.n_items + 3) / 4), dim3(256), 0, s, a);
}

void launch_select(int n_nodes, int ntests, const double* info, const int* thr, const int* k, TrBest* best, hipStream_t s) {
  hipLaunchKernelGGL(k_tr_select, dim3(n_nodes), dim3(256), 0, s, ntests, info, thr, k, best);
}

void launch_hp_items(const HpItemsArgs& a, int ntests, hipStream_t s) {
  hipLaunchKernelGGL(k_hp_items, dim3(ntests), dim3(256), 0, s, a);
}

void launch_hp_split(const HpSplitArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_hp_split, dim3(1), dim3(1024), 0, s, a);
}

void launch_partition(int n_nodes, const TrNode* nodes, const TrFeature* feats, const TrImage* imgs, const TrSample* samples,
                      const uint32_t* chan, const int32_t* list, int32_t* next, hipStream_t s) {
  hipLaunchKernelGGL(k_tr_partition, dim3(n_nodes), dim3(64), 0, s, nodes, feats, imgs, samples, chan, list, next);
}

}  // namespace ffd_train
