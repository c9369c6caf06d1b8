// ffd_kernels.hip — CDNA4 (gfx950) kernels of the analyzeFace hot path.
//
// Compiled with -ffp-contract=off: every float/double expression rounds exactly
// as written (explicit fmaf() only where the restatement defines a fused op), so
// the results are bit-identical to the CPU restatement in oracle/.
//
// Kernel map (reference -> kernel):
//   cvtColor + ROI + resize      FaceForest.cpp:195-204              k_gray_resize
//   Gabor filter2D + magnitude   FeatureChannelFactory.hpp:253-270   k_gabor7, k_gabor_sep<W>
//   normalize/convertTo/integral FeatureChannelFactory.hpp:271-286,  k_integral (+ gray, Sobel
//                                46-57, 120-141                       channels fused in)
//   Forest::evaluateMT           Forest.hpp:80-90, Tree.hpp:173-191,  k_traverse<HP/FFD>
//                                ImageSample.cpp:48-63
//   head-pose reduction + tree   face_utils.cpp:218-241,304-323,      k_hp_pose
//   selection                    FaceForest.cpp:214-250
//   vote filter                  face_utils.cpp:276-301               k_votes
//   MeanShift + rescale          MeanShift.hpp:41-135,                k_meanshift
//                                FaceForest.cpp:255-257
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <type_traits>
#include <cstdlib>

#include "../../include/ffd_numerics.h"
#include "ffd_device.hpp"
#include "ffd_kernels.hpp"

namespace ffd {

// ----------------------------------------------------------------- helpers --
__device__ __forceinline__ int reflect101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) {
    if (i < 0) i = -i;
    if (i >= n) i = 2 * n - 2 - i;
  }
  return i;
}

__device__ __forceinline__ int sat_u8(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }
__device__ __forceinline__ int sat_s16(int v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }

// cvRound(float): round half to even, NaN / out of range -> INT_MIN (cvtss2si).
__device__ __forceinline__ int cv_round(float v) {
  if (!(v >= -2147483648.0f && v < 2147483648.0f)) return (int)0x80000000;
  return (int)__builtin_rintf(v);
}

__device__ __forceinline__ uint8_t gray_px(const uint8_t* p) {  // BGR2GRAY, yuv_shift 14
  return (uint8_t)((p[0] * 1868 + p[1] * 9617 + p[2] * 4899 + (1 << 13)) >> 14);
}

// Map a dispatch block index to a logical block so that every XCD (blocks are dealt
// round-robin over the 8 XCDs) works on a contiguous logical range: consecutive
// faces' data then shares one XCD's L2.  Speed only, never correctness.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t nb) {
  uint32_t xcd = b & 7u, q = nb >> 3, r = nb & 7u;
  uint32_t start = xcd * q + (xcd < r ? xcd : r);
  return start + (b >> 3);
}

// ------------------------------------------------------ gray + ROI + resize --
// One workgroup per face; OpenCV 2.4.9 resize(INTER_LINEAR) 8U fixed-point path
// (HResizeLinear + VResizeLinearVec_32s8u SSE2 columns [0, xv) + scalar tail).
// STAGED (batches, source box <= the launch's dynamic LDS): the face's source box is first converted to gray into
// LDS (each source pixel once, coalesced BGR reads), then each thread owns one output column (its horizontal
// coefficients computed once) and walks every other row — the same expressions as the per-pixel form (round 6: C2
// 0.32 ms with each output pixel converting its four source pixels and dividing its index).
template <bool STAGED = false>
__global__ __launch_bounds__(256) void k_gray_resize(const FaceDesc* __restrict__ faces,
                                                     const uint8_t* __restrict__ images,
                                                     uint8_t* __restrict__ gray, int lds_cap) {
  extern __shared__ __attribute__((aligned(16))) uint8_t s_src[];
  const FaceDesc fd = faces[blockIdx.x];
  if (!fd.valid || fd.nochan) return;
  const uint8_t* img = images + fd.img_off;
  uint8_t* out = gray + fd.gray_off;
  const int sw = fd.bw, sh = fd.bh;
  const bool st = STAGED && sw * sh <= lds_cap;  // (a larger box: the per-pixel form below)
  if (st) {  // 8 pixels per thread per step, all their loads issued before the LDS stores (HBM latency, not bytes)
    const int n = sw * sh;
    for (int i0 = 0; i0 < n; i0 += 8 * 256) {
      uint8_t v[8];
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int i = min(i0 + k * 256 + (int)threadIdx.x, n - 1), y = i / sw, x = i - y * sw;
        v[k] = gray_px(img + (int64_t)(fd.by + y) * fd.img_stride + 3 * (fd.bx + x));
      }
#pragma unroll
      for (int k = 0; k < 8; k++)
        if (i0 + k * 256 + (int)threadIdx.x < n) s_src[i0 + k * 256 + threadIdx.x] = v[k];
    }
    __syncthreads();
  }
  auto G = [&](int y, int x) -> int {
    if (st) return s_src[y * sw + x];
    return gray_px(img + (int64_t)(fd.by + y) * fd.img_stride + 3 * (fd.bx + x));
  };
  // horizontal / vertical coefficients of the bilinear mode (OpenCV 2.4.9 fixed point, as oracle cv_resize)
  auto xcoef = [&](int dx, int& sx, int& a0, int& a1, bool& right) {
    float fx = (float)((dx + 0.5) * fd.scale_x - 0.5);
    sx = (int)floorf(fx);
    fx -= sx;
    if (sx < 0) fx = 0, sx = 0;
    right = false;
    if (sx + 1 >= sw) {
      right = true;
      if (sx >= sw - 1) fx = 0, sx = sw - 1;
    }
    a0 = sat_s16(cv_round((1.f - fx) * 2048.f));
    a1 = sat_s16(cv_round(fx * 2048.f));
  };
  auto pixel = [&](int dy, int dx, int sx, int a0, int a1, bool right) -> int {
    if (fd.mode == 0) return G(dy, dx);
    if (fd.mode == 2)
      return (G(2 * dy, 2 * dx) + G(2 * dy, 2 * dx + 1) + G(2 * dy + 1, 2 * dx) + G(2 * dy + 1, 2 * dx + 1) + 2) >> 2;
    float fy = (float)((dy + 0.5) * fd.scale_y - 0.5);
    int sy = (int)floorf(fy);
    fy -= sy;
    int b0 = sat_s16(cv_round((1.f - fy) * 2048.f)), b1 = sat_s16(cv_round(fy * 2048.f));
    int y0 = min(max(sy, 0), sh - 1), y1 = min(max(sy + 1, 0), sh - 1);
    int r0, r1;
    if (right) {
      r0 = G(y0, sx) * 2048;
      r1 = G(y1, sx) * 2048;
    } else {
      r0 = G(y0, sx) * a0 + G(y0, sx + 1) * a1;
      r1 = G(y1, sx) * a0 + G(y1, sx + 1) * a1;
    }
    if (dx < fd.xv) {
      int s0 = max(-32768, min(32767, r0 >> 4)), s1 = max(-32768, min(32767, r1 >> 4));
      int m = max(-32768, min(32767, ((s0 * b0) >> 16) + ((s1 * b1) >> 16)));
      m = max(-32768, min(32767, m + 2)) >> 2;
      return sat_u8(m);
    }
    return sat_u8((b0 * r0 + b1 * r1 + (1 << 21)) >> 22);
  };
  if (st) {  // a thread per output column (W <= 125 < 128), two rows per pass
    const int dx = threadIdx.x & 127;
    if (dx >= fd.W) return;
    int sx = 0, a0 = 0, a1 = 0;
    bool right = false;
    if (fd.mode == 1) xcoef(dx, sx, a0, a1, right);
    for (int dy = threadIdx.x >> 7; dy < fd.H; dy += 2) out[dy * PITCH + dx] = (uint8_t)pixel(dy, dx, sx, a0, a1, right);
    return;
  }
  for (int i = blockIdx.y * blockDim.x + threadIdx.x; i < fd.W * fd.H; i += gridDim.y * blockDim.x) {
    int dy = i / fd.W, dx = i % fd.W;
    int sx = 0, a0 = 0, a1 = 0;
    bool right = false;
    if (fd.mode == 1) xcoef(dx, sx, a0, a1, right);
    out[dy * PITCH + dx] = (uint8_t)pixel(dy, dx, sx, a0, a1, right);
  }
}

// ---------------------------------------------------------------- integral --
// One wave per (face, channel): the wave walks the rows top to bottom; lane l owns image columns
// 2l, 2l+1, keeps their running column sums, and a 64-lane prefix scan turns them into integral
// rows; lane l writes integral entries 2l, 2l+1 as one aligned u32 (entry 2l = exclusive prefix,
// 2l+1 = + column 2l).  Integer-exact, so order does not matter; stored modulo 2^16 (rect_mean16).
__device__ __forceinline__ int chan_value(int c, const uint8_t* g, int W, int H, int y, int x) {
  if (x >= W) return 0;
  if (c == 0) return g[y * PITCH + x];
  int ym = reflect101(y - 1, H), yp = reflect101(y + 1, H), xm = reflect101(x - 1, W), xp = reflect101(x + 1, W);
  auto I = [&](int yy, int xx) { return (int)g[yy * PITCH + xx]; };
  int v;
  if (c == 36)  // Sobel(0,1): d/dy
    v = (I(yp, xm) + 2 * I(yp, x) + I(yp, xp)) - (I(ym, xm) + 2 * I(ym, x) + I(ym, xp));
  else          // Sobel(1,0): d/dx
    v = (I(ym, xp) + 2 * I(y, xp) + I(yp, xp)) - (I(ym, xm) + 2 * I(y, xm) + I(yp, xm));
  return sat_u8(v);
}

// Inclusive prefix sum over the 64 lanes of a wave with DPP: row_shr 1, 2, 4, 8 within each row of
// 16 lanes, then row_bcast:15 (rows 1, 3 add lane 15 of the row before) and row_bcast:31 (rows 2, 3
// add lane 31).  Integer adds: the order does not matter.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false); // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false); // row_bcast:31
  return v;
}

// The scan of one channel by one wave.  value(y, b) returns the u8 values of columns 2l, 2l+1 of
// row y for b = 0..RB-1 batches (all of a batch's loads are issued before its scans).
// One integral row from this row's values v0, v1 (columns 2l, 2l + 1): exact (c0, c1: running column
// sums, the row's entries by a prefix scan of them) or, for a float-integral face (FaceDesc::fint), as
// OpenCV's integral_ in float (f0, f1: the entries of the row above; + this row's prefix s, rounded):
// the same values until one reaches 2^24.  Returns entries 2l | 2l + 1 << 16, modulo 2^16 each.
__device__ __forceinline__ uint32_t integral_row(bool fl, uint32_t v0, uint32_t v1, uint32_t& c0, uint32_t& c1,
                                                 float& f0, float& f1) {
  if (!fl) {
    c0 += v0;
    c1 += v1;
    const uint32_t s2 = c0 + c1;
    const uint32_t excl = wave_incl_scan(s2) - s2;
    return (excl & 0xFFFFu) | ((excl + c0) << 16);
  }
  const uint32_t p = v0 + v1, s = wave_incl_scan(p) - p;  // this row's prefix up to column 2l - 1 (exact)
  f0 = f0 + (float)s;
  f1 = f1 + (float)(s + v0);
  return ((uint32_t)f0 & 0xFFFFu) | ((uint32_t)f1 << 16);
}

template <int RB = 8, class RowFn>
__device__ __forceinline__ void integral_scan(uint16_t* __restrict__ out, int W, int H, int lane, bool fl, RowFn row_values) {
  for (int x = lane; x <= W; x += 64) out[x] = 0;  // row 0 of the integral image
  uint32_t c0 = 0, c1 = 0;
  float f0 = 0.f, f1 = 0.f;
  for (int y0 = 0; y0 < H; y0 += RB) {
    uint32_t v0[RB], v1[RB];
    row_values(y0, v0, v1);
#pragma unroll
    for (int b = 0; b < RB; b++) {
      if (y0 + b >= H) break;
      uint32_t* r = reinterpret_cast<uint32_t*>(out + (int64_t)(y0 + b + 1) * PITCH);
      // entries >= W+1 land in the row's pitch padding (never read by a patch)
      r[lane] = integral_row(fl, v0[b], v1[b], c0, c1, f0, f1);
    }
  }
}

// gray (channel 0) and the two Sobel channels (36 d/dy, 37 d/dx); the 35 Gabor channels are
// integrated by the Gabor kernels themselves.  One 4-wave workgroup per face (the 4th wave idles).
// STAGE (small batches): the face's gray rows are first copied to LDS by all four waves, so the three
// sequential scans read their values at LDS rather than L2 latency.
#ifndef FFD_SOBEL_ROWS
#define FFD_SOBEL_ROWS 1  // Sobel values from each batch's source rows read once (0: six neighbour reads per value)
#endif
#ifndef FFD_INTEGRAL_STAGE_ALL
#define FFD_INTEGRAL_STAGE_ALL 1  // batches too stage the face's gray rows in LDS (0: small batches only)
#endif
// One of the non-Gabor integral channels (c = 0 gray, 36 Sobel d/dy, 37 Sobel d/dx) of a face, by one wave; g: the
// face's gray rows (global, or staged in LDS).
__device__ __forceinline__ void integral_channel(const FaceDesc& fd, const uint8_t* g, uint16_t* __restrict__ chan,
                                                 int c, int lane) {
  const int W = fd.W, H = fd.H, x0 = 2 * lane;
  uint16_t* out = chan + fd.ch_off + (int64_t)c * fd.plane;
  if (c == 0 || !FFD_SOBEL_ROWS) {
    integral_scan(out, W, H, lane, fd.fint != 0, [&](int y0, uint32_t* v0, uint32_t* v1) {
#pragma unroll
      for (int b = 0; b < 8; b++) {
        const int y = min(y0 + b, H - 1);
        v0[b] = (uint32_t)chan_value(c, g, W, H, y, x0);
        v1[b] = (uint32_t)chan_value(c, g, W, H, y, x0 + 1);
      }
    });
    return;
  }
  // Sobel (chan_value's arithmetic): a batch of 8 rows reads its 10 source rows (reflect-101) once, at the lane's
  // four columns x0 - 1, x0, x0 + 1, x0 + 2 (reflect-101), instead of six neighbours per value (12 per row)
  const int xs = min(x0, W - 1);  // (lanes past the face read valid columns; their values are 0)
  const int ca = reflect101(xs - 1, W), cb = xs, cc = reflect101(xs + 1, W), cd = reflect101(xs + 2, W);
  const bool in0 = x0 < W, in1 = x0 + 1 < W;
  integral_scan(out, W, H, lane, fd.fint != 0, [&](int y0, uint32_t* v0, uint32_t* v1) {
    int A[10], B[10], C[10], D[10];
#pragma unroll
    for (int k = 0; k < 10; k++) {
      const uint8_t* row = g + reflect101(min(y0 - 1 + k, H), H) * PITCH;  // (rows past H - 1: unused values)
      A[k] = row[ca];
      B[k] = row[cb];
      C[k] = row[cc];
      D[k] = row[cd];
    }
#pragma unroll
    for (int b = 0; b < 8; b++) {  // rows ym = b, y = b + 1, yp = b + 2 of the arrays
      int s0, s1;
      if (c == 36) {  // Sobel(0,1): d/dy
        s0 = (A[b + 2] + 2 * B[b + 2] + C[b + 2]) - (A[b] + 2 * B[b] + C[b]);
        s1 = (B[b + 2] + 2 * C[b + 2] + D[b + 2]) - (B[b] + 2 * C[b] + D[b]);
      } else {        // Sobel(1,0): d/dx
        s0 = (C[b] + 2 * C[b + 1] + C[b + 2]) - (A[b] + 2 * A[b + 1] + A[b + 2]);
        s1 = (D[b] + 2 * D[b + 1] + D[b + 2]) - (B[b] + 2 * B[b + 1] + B[b + 2]);
      }
      v0[b] = in0 ? (uint32_t)sat_u8(s0) : 0u;
      v1[b] = in1 ? (uint32_t)sat_u8(s1) : 0u;
    }
  });
}

#ifndef FFD_GS_CPT2_MASK
#define FFD_GS_CPT2_MASK 12  // bit nu (2: 13x13, 3: 19x19, 4: 25x25): the batch instance with 2 columns per H-pass thread (25x25: spills at 128 VGPRs, 1.93 -> 2.68 ms)
#endif
#ifndef FFD_GS_CPT2S_MASK
#define FFD_GS_CPT2S_MASK 18  // bit nu: the 2-column instance in 256-thread workgroups (4-row bands; 25x25 1.91 -> 1.74, 9x9 1.20 -> 1.16 ms)
#endif
#ifndef FFD_GS_CPT2S_WAVES
#define FFD_GS_CPT2S_WAVES 3  // ... its waves per SIMD (3: <= 168 VGPRs, three workgroups per CU)
#endif
#ifndef FFD_GS_CPT2_WAVES
#define FFD_GS_CPT2_WAVES 4  // ... its waves per SIMD (4: <= 128 VGPRs, two 512-thread workgroups per CU)
#endif
#ifndef FFD_GABOR_BAND_ALL
#define FFD_GABOR_BAND_ALL 0  // 1: every face through the band-staged (TALL) instance (LDS 66 -> 49 KB per workgroup)
#endif

template <bool STAGE>
__global__ __launch_bounds__(256) void k_integral(const FaceDesc* __restrict__ faces,
                                                  const uint8_t* __restrict__ gray,
                                                  uint16_t* __restrict__ chan) {
  extern __shared__ __attribute__((aligned(16))) uint8_t s_gray[];  // STAGE: H x PITCH
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const FaceDesc fd = faces[blockIdx.x];
  if (!fd.valid || fd.nochan) return;
  const int H = fd.H;
  const uint8_t* g = gray + fd.gray_off;
  if (STAGE) {
    for (int i = threadIdx.x; i < H * (PITCH / 16); i += 256)
      reinterpret_cast<uint4*>(s_gray)[i] = reinterpret_cast<const uint4*>(g)[i];
    __syncthreads();
    g = s_gray;
  }
  if (wv >= 3) return;
  integral_channel(fd, g, chan, wv == 0 ? 0 : 35 + wv, lane);
}

// ------------------------------------------------------------------ Gabor --
typedef float f2 __attribute__((ext_vector_type(2)));

// Face-wide min / max of one scale's 7 magnitude planes -> cv::normalize(NORM_MINMAX, 0, 1) +
// convertTo(CV_8U, 255) (FeatureChannelFactory.hpp:271-286): quantise (v*scale + shift, *255,
// cvRound, saturate) and integrate the 7 channels, one wave per channel, reading the magnitudes
// back from L2.  mn / mx: this thread's minimum and maximum of the magnitudes' bits (unsigned
// order == float order for m >= +0).  Every magnitude store of the workgroup precedes
// the first barrier here.
template <int NWV>
__device__ __forceinline__ void gabor_minmax_scale(uint32_t (&mn)[7], uint32_t (&mx)[7], float* s_sf, float* s_hf) {
  __shared__ uint32_t red[NWV][14];
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
#pragma unroll
  for (int o = 0; o < 7; o++) {
#pragma unroll
    for (int sh = 32; sh >= 1; sh >>= 1) {
      mn[o] = min(mn[o], (uint32_t)__shfl_xor((int)mn[o], sh));
      mx[o] = max(mx[o], (uint32_t)__shfl_xor((int)mx[o], sh));
    }
  }
  if (ln == 0) {
#pragma unroll
    for (int o = 0; o < 7; o++) { red[wv][o] = mn[o]; red[wv][7 + o] = mx[o]; }
  }
  __syncthreads();
  if (threadIdx.x < 7) {
    const int o = threadIdx.x;
    uint32_t a = red[0][o], b = red[0][7 + o];
    for (int w = 1; w < NWV; w++) { a = min(a, red[w][o]); b = max(b, red[w][7 + o]); }
    const double smin = (double)__uint_as_float(a), smax = (double)__uint_as_float(b);
    const double dmin = 0, dmax = 1;
    const double scale = (dmax - dmin) * (smax - smin > 2.220446049250313e-16 ? 1. / (smax - smin) : 0);
    const double shift = dmin - smin * scale;
    s_sf[o] = (float)scale;
    s_hf[o] = (float)shift;
  }
  __syncthreads();
}

// convertTo(CV_8U, 255) of a normalised magnitude (FeatureChannelFactory.hpp:276):
// saturate(cvRound(v * 255 + 0)).  "+ 0" only turns -0 into +0, which cvRound maps to 0 either way,
// and v * 255 lies in [-1, 256] for every magnitude of the plane (m in [min, max]), where cvRound's
// out-of-range test never fires: both are left out (the values are the same for every input).
__device__ __forceinline__ uint32_t gabor_quantise(float m, float sf, float hf) {
  return (uint32_t)sat_u8((int)__builtin_rintf((m * sf + hf) * 255.f));
}

// Correctly rounded sqrt of a magnitude's squared norm s (finite, >= +0), branch-free: the compiler's
// expansion of sqrtf (v_sqrt_f32, then the two residual tests with its neighbours) without its
// subnormal scaling and its class test.  Both are identities for s = +0 (the rm residual is NaN, the rp
// residual +0) and for s >= 2^-96 (no scaling applies), so mag_sqrt(s) == sqrtf(s) there.  For
// 0 < s < 2^-96 (both |re| and |im| below 2^-48: not met by real faces) it may differ: the Gabor
// kernels flag such a face (mag_tiny) and their EXACT instance recomputes it with sqrtf.
__device__ __forceinline__ float mag_sqrt(float s) {
  const float r = __builtin_amdgcn_sqrtf(s);
  const float rm = __uint_as_float(__float_as_uint(r) - 1u), rp = __uint_as_float(__float_as_uint(r) + 1u);
  const float r1 = __builtin_fmaf(-rm, r, s) <= 0.f ? rm : r;
  return __builtin_fmaf(-rp, r, s) > 0.f ? rp : r1;
}
// running minimum of bits(s) - 1: below 0x0F7FFFFF iff some 0 < s < 2^-96 was seen
__device__ __forceinline__ void mag_tiny_update(uint32_t& t, float s) { t = min(t, __float_as_uint(s) - 1u); }
template <bool EXACT, bool FAST>
__device__ __forceinline__ float mag_of(float s, uint32_t& tiny) {
  if (EXACT || !FAST) return __builtin_sqrtf(s);
  mag_tiny_update(tiny, s);
  return mag_sqrt(s);
}
// fast instance: record whether the face needs the exact instance (one workgroup-wide vote, after
// the compute phase); every valid face's flag is written, so the array needs no clearing
template <bool EXACT>
__device__ __forceinline__ void mag_flag(uint32_t tiny, int* __restrict__ redo, int force) {
  if (EXACT) return;
  const int any = __syncthreads_or(tiny < 0x0F7FFFFFu || force ? 1 : 0);
  if (threadIdx.x == 0) redo[blockIdx.x] = any;
}

template <int NWV>
__device__ __forceinline__ void gabor_normalise_integrate(const FaceDesc& fd, int nu, uint32_t (&mn)[7],
                                                          uint32_t (&mx)[7], const float* __restrict__ mag,
                                                          uint16_t* __restrict__ chan) {
  __shared__ float s_sf[7], s_hf[7];
  gabor_minmax_scale<NWV>(mn, mx, s_sf, s_hf);
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int x0 = 2 * lane, FW = fd.W, FH = fd.H;
  // Software-pipelined read-back: the magnitudes of rows [y0 + RB, y0 + 2RB) are in flight while rows
  // [y0, y0 + RB) are quantised and scanned (two register buffers), so the L2 / Infinity-Cache
  // latency of the read-back is paid once per plane instead of once per batch.
  constexpr int RB = 16;
  typedef float2 rowbuf[RB];
  for (int o = wv; o < 7; o += NWV) {
    const float sf = s_sf[o], hf = s_hf[o];
    const float* m = mag + fd.mag_off + (int64_t)(nu * 7 + o) * FH * PITCH + x0;
    uint16_t* out = chan + fd.ch_off + (int64_t)(1 + nu * 7 + o) * fd.plane;
    for (int x = lane; x <= FW; x += 64) out[x] = 0;  // row 0 of the integral image
    uint32_t c0 = 0, c1 = 0;
    float f0 = 0.f, f1 = 0.f;
    const bool fl = fd.fint != 0;
    auto load = [&](int y0, rowbuf& mv) {
#pragma unroll
      for (int b = 0; b < RB; b++)
        mv[b] = (y0 + b < FH) ? *reinterpret_cast<const float2*>(&m[(y0 + b) * PITCH]) : make_float2(0.f, 0.f);
    };
    auto scan = [&](int y0, const rowbuf& mv) {
#pragma unroll
      for (int b = 0; b < RB; b++) {
        if (y0 + b >= FH) break;
        const uint32_t q0 = (x0 < FW) ? gabor_quantise(mv[b].x, sf, hf) : 0u;
        const uint32_t q1 = (x0 + 1 < FW) ? gabor_quantise(mv[b].y, sf, hf) : 0u;
        // entries >= W+1 land in the row's pitch padding (never read by a patch)
        reinterpret_cast<uint32_t*>(out + (int64_t)(y0 + b + 1) * PITCH)[lane] = integral_row(fl, q0, q1, c0, c1, f0, f1);
      }
    };
    rowbuf A, B;
    load(0, A);
    for (int y0 = 0; y0 < FH; y0 += 2 * RB) {
      if (y0 + RB < FH) load(y0 + RB, B);
      scan(y0, A);
      if (y0 + RB >= FH) break;
      if (y0 + 2 * RB < FH) load(y0 + 2 * RB, A);
      scan(y0 + RB, B);
    }
  }
}

// running min / max of a plane's magnitudes as their bits (unsigned order == float order for m >= +0).
// MASK: pixels outside the face (in == false) enter as the neutral elements (all ones / zero), four
// ALU operations with no select; else a predicated update.  Which form a kernel uses is decided per
// Gabor scale by measurement (the register allocator's SGPR spills differ, k_gabor_sep below).
template <bool MASK>
__device__ __forceinline__ void minmax_update(uint32_t& mn, uint32_t& mx, float m, bool in) {
  const uint32_t bits = __float_as_uint(m);
  if (MASK) {
    const uint32_t im = in ? 0xFFFFFFFFu : 0u;
    mn = min(mn, bits | ~im);
    mx = max(mx, bits & im);
  } else if (in) {
    mn = min(mn, bits);
    mx = max(mx, bits);
  }
}

// Banded (SPLIT) Gabor instances for small batches: a face's bands (sep) or tiles (7x7) are spread over
// gridDim.y workgroups, each of which writes its magnitudes and folds its min / max (and the fast
// instance's tiny-magnitude vote) into the face's 16-word slot mm = [~min x 7, max x 7, flag, arrivals]
// with device-scope atomics; the workgroup that arrives last takes the totals (resetting the slot to
// zero for the next launch) and runs the normalise / integrate epilogue over the whole face.
// Returns true in that workgroup only; its thread 0 then holds the face's min / max in mn / mx.
template <bool EXACT>
__device__ __forceinline__ bool split_finish(uint32_t (&mn)[7], uint32_t (&mx)[7], uint32_t tiny, int force,
                                             uint32_t* __restrict__ mm, int nwg, int* __restrict__ redo_f) {
  __shared__ uint32_t s_mm[16];
  __shared__ int s_last;
  const int tid = threadIdx.x, lane = tid & 63;
  if (tid < 16) s_mm[tid] = 0u;
  __syncthreads();
#pragma unroll
  for (int o = 0; o < 7; o++) {
    uint32_t a = mn[o], b = mx[o];
#pragma unroll
    for (int sh = 32; sh >= 1; sh >>= 1) {
      a = min(a, (uint32_t)__shfl_xor((int)a, sh));
      b = max(b, (uint32_t)__shfl_xor((int)b, sh));
    }
    if (lane == 0) {
      atomicMax(&s_mm[o], ~a);
      atomicMax(&s_mm[7 + o], b);
    }
  }
  const int any = EXACT ? 0 : __syncthreads_or(tiny < 0x0F7FFFFFu || force ? 1 : 0);
  __syncthreads();
  if (tid < 14 && s_mm[tid]) atomicMax(&mm[tid], s_mm[tid]);
  if (tid == 14 && any) atomicOr(&mm[14], 1u);
  __threadfence();  // this workgroup's magnitudes and slot updates before its arrival
  __syncthreads();
  if (tid == 0) s_last = atomicAdd(&mm[15], 1u) == (uint32_t)(nwg - 1) ? 1 : 0;
  __syncthreads();
  if (!s_last) return false;
  __threadfence();  // every other workgroup's magnitudes are visible from here
  if (tid < 16) s_mm[tid] = atomicExch(&mm[tid], 0u);
  __syncthreads();
#pragma unroll
  for (int o = 0; o < 7; o++) {
    mn[o] = tid == 0 ? ~s_mm[o] : 0xFFFFFFFFu;
    mx[o] = tid == 0 ? s_mm[7 + o] : 0u;
  }
  if (!EXACT && tid == 0) *redo_f = s_mm[14] != 0u ? 1 : 0;
  return true;
}

// 7x7 (scale 0): OpenCV 2.4.9's direct Filter2D (49 taps < dft_filter_size 50), restated bit-exactly.
// Coefficients (host-built from createKernel, FeatureChannelFactory.hpp:186-251), 16 floats per tap
// in row-major order: [re0, im0, re1, im1, ..., re6, im6, 0, 0].
// One 512-thread workgroup computes 64x32 output tiles of one face for the 7 orientations from an
// LDS copy of the (reflect-101 padded) input tile; each thread owns 4 horizontally adjacent pixels,
// the (re, im) pairs accumulate as packed mul + add (s = 0; s += k*p, no FMA) whose coefficient
// operands are wave-uniform scalar loads (SGPR pairs).
#ifndef FFD_G7_ROWREG
#define FFD_G7_ROWREG 1  // 0: per-tap LDS reads (2.22 ms at C2); 1: each tap row's 10 inputs read once into registers (7 taps unrolled)
#endif
constexpr int GB_TX = 64, GB_TY = 32, GB_THREADS = 512;

template <bool EXACT, bool SPLIT>
__global__ __launch_bounds__(GB_THREADS) void k_gabor7(const FaceDesc* __restrict__ faces,
                                                       const uint8_t* __restrict__ gray,
                                                       const float4* __restrict__ coef_g,
                                                       float* __restrict__ mag,
                                                       uint16_t* __restrict__ chan, int* __restrict__ redo, int force,
                                                       uint32_t* __restrict__ split_mm) {
  constexpr int R = 3;
  // row stride (floats) == 1 mod 4: the 4 rows a 32-lane group touches fall on disjoint banks
  constexpr int LW = ((GB_TX + 2 * R + 3) / 4) * 4 + 1;
  constexpr int LH = GB_TY + 2 * R;
  __shared__ float tile[LH * LW];
  const FaceDesc fd = faces[blockIdx.x];
  if (!fd.valid || fd.nochan) return;
  if (EXACT && !redo[blockIdx.x]) return;  // the fast instance's mag_sqrt was exact for this face
  uint32_t tiny = 0xFFFFFFFFu;
  const int tiles_x = (fd.W + GB_TX - 1) / GB_TX, tiles = tiles_x * ((fd.H + GB_TY - 1) / GB_TY);
  int tl0 = 0, tl1 = tiles, nwg = 1;
  if (SPLIT) {  // this workgroup's share of the face's tiles
    const int per = (tiles + gridDim.y - 1) / gridDim.y;
    nwg = (tiles + per - 1) / per;
    if ((int)blockIdx.y >= nwg) return;
    tl0 = blockIdx.y * per;
    tl1 = min(tiles, tl0 + per);
  }
  const uint8_t* g = gray + fd.gray_off;
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  uint32_t mn[7], mx[7];
#pragma unroll
  for (int o = 0; o < 7; o++) { mn[o] = 0xFFFFFFFFu; mx[o] = 0u; }
#pragma unroll 1
  for (int tl = tl0; tl < tl1; tl++) {
    const int tx0 = (tl % tiles_x) * GB_TX, ty0 = (tl / tiles_x) * GB_TY;
    __syncthreads();  // the previous tile's reads of `tile` are done
    for (int i = threadIdx.x; i < LH * (GB_TX + 2 * R); i += GB_THREADS) {
      const int ly = i / (GB_TX + 2 * R), lx = i % (GB_TX + 2 * R);
      const int y = reflect101(ty0 - R + ly, fd.H), x = reflect101(tx0 - R + lx, fd.W);
      tile[ly * LW + lx] = (float)g[y * PITCH + x];
    }
    __syncthreads();
    // wave w covers threads tx in [8*(w&1), +8) x ty in [8*(w>>1), +8); 4 px per thread
    const int tx = (wv & 1) * 8 + (ln & 7), ty = (wv >> 1) * 8 + (ln >> 3);
    // acc[k][o] = (re, im): one v_pk_mul + v_pk_add per (pixel, orientation), each half of
    // which is exactly the scalar mul + add of the restatement
    f2 acc[4][7];
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int o = 0; o < 7; o++) acc[k][o] = f2{0.f, 0.f};
    // centre pixel (ty, 4tx + k) sits at tile (ty + R, 4tx + R + k)
    const float* ctr = &tile[(ty + R) * LW + 4 * tx + R];
#if FFD_G7_ROWREG
    // a row's 10 input values once into registers, its 7 taps from them (same tap order)
#pragma unroll 1
    for (int r = 0; r < 7; r++) {
      const float* prow = ctr + (r - 3) * LW - 3;
      float pv[10];
#pragma unroll
      for (int j = 0; j < 10; j++) pv[j] = prow[j];
#pragma unroll
      for (int dxi = 0; dxi < 7; dxi++) {
        const int t = r * 7 + dxi;
        const float4 c0 = coef_g[t * 4 + 0], c1 = coef_g[t * 4 + 1], c2 = coef_g[t * 4 + 2], c3 = coef_g[t * 4 + 3];
        const f2 c[7] = {f2{c0.x, c0.y}, f2{c0.z, c0.w}, f2{c1.x, c1.y}, f2{c1.z, c1.w},
                         f2{c2.x, c2.y}, f2{c2.z, c2.w}, f2{c3.x, c3.y}};
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const f2 pp = f2{pv[dxi + k], pv[dxi + k]};
#pragma unroll
          for (int o = 0; o < 7; o++) acc[k][o] = acc[k][o] + c[o] * pp;
        }
      }
    }
#else
#pragma unroll 1
    for (int r = 0; r < 7; r++) {
      const float* prow = ctr + (r - 3) * LW;
#pragma unroll 1
      for (int dxi = 0; dxi < 7; dxi++) {
        const float* pa = prow + (dxi - 3);
        const int t = r * 7 + dxi;
        const float4 c0 = coef_g[t * 4 + 0], c1 = coef_g[t * 4 + 1], c2 = coef_g[t * 4 + 2], c3 = coef_g[t * 4 + 3];
        const f2 c[7] = {f2{c0.x, c0.y}, f2{c0.z, c0.w}, f2{c1.x, c1.y}, f2{c1.z, c1.w},
                         f2{c2.x, c2.y}, f2{c2.z, c2.w}, f2{c3.x, c3.y}};
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const float p = pa[k];
          const f2 pp = f2{p, p};
#pragma unroll
          for (int o = 0; o < 7; o++) acc[k][o] = acc[k][o] + c[o] * pp;
        }
      }
    }
#endif
    const int x0 = tx0 + 4 * tx, y = ty0 + ty;
#pragma unroll
    for (int o = 0; o < 7; o++) {
      float m4[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const float i2 = acc[k][o].y * acc[k][o].y, r2 = acc[k][o].x * acc[k][o].x;
        m4[k] = mag_of<EXACT, true>(i2 + r2, tiny);
        minmax_update<true>(mn[o], mx[o], m4[k], (x0 + k) < fd.W && y < fd.H);
      }
      if (y < fd.H)  // columns >= W land in the row's pitch padding, never read
        *reinterpret_cast<float4*>(&mag[fd.mag_off + ((int64_t)o * fd.H + y) * PITCH + x0]) =
            make_float4(m4[0], m4[1], m4[2], m4[3]);
    }
  }
  if (SPLIT) {
    if (!split_finish<EXACT>(mn, mx, tiny, force, split_mm + ((int64_t)blockIdx.x * 5 + 0) * 16, nwg,
                             redo + blockIdx.x))
      return;
  } else {
    mag_flag<EXACT>(tiny, redo, force);
  }
  gabor_normalise_integrate<GB_THREADS / 64>(fd, 0, mn, mx, mag, chan);
}

// Scales 1..4 (9x9 .. 25x25): the separable definition of include/ffd_gabor.h, in the operation
// order of oracle/ffd_oracle.cpp gabor_sep_mag.  One 256-thread workgroup per face walks bands of
// GS_BY output rows:
//   stage   the band's gray rows [y0-R, y0+BY+R) x padded columns [-R, W+R) (reflect-101) as floats;
//   V pass  per (row, padded column): Vg and (Vc_q, Vs_q), q = 1..4 (folded taps, packed FMAs);
//   H pass  per (row, 4 adjacent columns): the 7 orientations' (re, im) as packed FMAs over the
//           V planes (taps -R..R), the DC term, magnitudes to HBM, running min / max.
// V planes sit in LDS "quad-split": padded column cc at (cc & 3) * QS + (cc >> 2), so the 32 lanes
// of an H-pass row reading column 4*cq + u hit 32 consecutive words (conflict-free ds_read_b64).
// Coefficient block (floats, host-built by ffd_engine build_gabor from ffd_gabor_sep):
//   [0]                 c
//   V_OFF + 12 t        t = 0..R: g, 0, (vc_q, vs_q) q = 1..4, 0, 0
//   H_OFF + 16 (t + R)  t = -R..R: (hc0, hs0), (g, g), then for p = 1..3 (hc_p, hc_p, hs_p, hs_p)
//                       [hs_p(t) odd in t]
constexpr int GS_THREADS = 256, GS_BY = 8;
#ifndef FFD_GS_QSPLIT
#define FFD_GS_QSPLIT 1  // k_gabor_sep: V / H passes in two plane halves (LDS 66 -> 47 KB at 25x25: 3 WGs per CU)
#endif
constexpr bool GS_QSPLIT = FFD_GS_QSPLIT;
#ifndef FFD_GABOR_SPLIT_MAX
#define FFD_GABOR_SPLIT_MAX 16  // batches of up to 16 faces: banded Gabor instances (SPLIT)
#endif
#ifndef FFD_GABOR_SPLIT_WG
#define FFD_GABOR_SPLIT_WG 16   // workgroups per face and scale in the banded instances
#endif


// CPT: output columns per H-pass thread (4: 256-thread workgroups; 2: 512 threads, half the accumulators per thread)
template <int R, int CPT = 4> struct GSep {
  static constexpr int GP = (PITCH + 2 * R + 3) / 4 * 4;  // padded gray row pitch (bytes)
  static constexpr int LC = CPT == 4 ? 2 : 1;             // log2(CPT)
  // V values "CPT-split": padded column cc at slot (cc % CPT) * QS + cc / CPT, so the lanes of an H-pass row
  // (column groups cq, cq + 1, ...) reading column CPT * cq + u hit consecutive words
  static constexpr int QS = 128 / CPT + ((CPT - 1 + 2 * R) >> LC);
  static constexpr int VP = CPT * QS;                     // V row pitch (elements) >= W + 2R
  static constexpr int SC = GP;                           // staging / V-pass column range
  static constexpr int V_OFF = 4, H_OFF = 4 + 12 * (R + 1);
};
// threads of a k_gabor_sep workgroup: BY rows x 128 / CPT column groups
__host__ __device__ constexpr int gs_threads(int cpt, int by = 8) { return by * 128 / cpt; }

// TALL: the instance for faces taller than MAX_FACE_H (box aspect h/w > 4.8), whose padded face does not
// fit the LDS: each band stages only its GS_BY + 2R rows (4x re-staging at 25x25; such faces are rare).
// Each instance skips the other's faces.
template <int W, bool EXACT, bool TALL, bool SPLIT = false, int CPT = 4, int BY = GS_BY>
__global__ __launch_bounds__(gs_threads(CPT, BY))
__attribute__((amdgpu_waves_per_eu(CPT == 2 ? (BY == GS_BY ? FFD_GS_CPT2_WAVES : FFD_GS_CPT2S_WAVES) : 1)))
void k_gabor_sep(const FaceDesc* __restrict__ faces,
                                                          const uint8_t* __restrict__ gray,
                                                          const float* __restrict__ coef,
                                                          float* __restrict__ mag,
                                                          uint16_t* __restrict__ chan, int* __restrict__ redo, int force,
                                                          uint32_t* __restrict__ split_mm) {
  static_assert(!(TALL && SPLIT), "tall faces are not banded across workgroups");
  constexpr int R = (W - 1) / 2;
  using C = GSep<R, CPT>;
  constexpr int GS_THREADS = gs_threads(CPT, BY);
  static_assert(CPT == 4 || (CPT == 2 && !TALL && !SPLIT), "2-column threads: the batch instance only");
  static_assert(GS_BY % BY == 0, "bands: the staged rows are allocated for whole bands of 8 rows");
  constexpr int NU = W == 9 ? 1 : W == 13 ? 2 : W == 19 ? 3 : 4;
  // magnitude sqrt / min-max forms per scale (r2e, C2, ms): 25x25 sqrtf + masked min-max 1.88 (both
  // compiler forms 1.93, both fast 2.04: SGPR spills); 19x19 both fast 1.63 (1.72); 13x13 / 9x9
  // mag_sqrt + predicated min-max 1.44 / 1.30 (1.54 / 1.34; masked: SGPR spills, 2.8 / 1.7)
  constexpr bool GS_FAST = W != 25, GS_MASK = W == 25 || W == 19;
  extern __shared__ __attribute__((aligned(16))) uint8_t gface[];  // (H + 2R) x GP reflect-101 padded face
  __shared__ float vg[BY * C::VP];
  // QS: the V / H passes in two plane halves (half the V-plane LDS, fewer live registers): measured faster
  // for 9x9 only (1.34 -> 1.16 ms; 13x13 / 19x19 even, 25x25 1.96 -> 2.43)
  constexpr bool QS = GS_QSPLIT && W == 9 && CPT == 4;
  __shared__ f2 vq[QS ? 2 : 4][BY * C::VP];
  const FaceDesc fd = faces[blockIdx.x];
  if (!fd.valid || fd.nochan || ((FFD_GABOR_BAND_ALL && !SPLIT) ? !TALL : (fd.H > MAX_FACE_H) != TALL)) return;
  if (EXACT && !redo[blockIdx.x]) return;  // the fast instance's mag_sqrt was exact for this face
  uint32_t tiny = 0xFFFFFFFFu;
  const int FW = fd.W, FH = fd.H, NPC = FW + 2 * R;
  const uint8_t* g = gray + fd.gray_off;
  const float* cv = coef + C::V_OFF;
  const float* chh = coef + C::H_OFF;
  const float cdc = coef[0];
  const int tid = threadIdx.x;
  uint32_t mn[7], mx[7];
#pragma unroll
  for (int o = 0; o < 7; o++) { mn[o] = 0xFFFFFFFFu; mx[o] = 0u; }

  // the reflect-101 padded face rows [r0, r0 + rows) (padded-row index: face row + R) to LDS rows
  // [0, rows): (row, 4-column group) items, u32 LDS stores
  auto stage_rows = [&](int r0, int rows) {
    constexpr int NQ = C::GP / 4;
    for (int i = tid; i < rows * NQ; i += GS_THREADS) {
      const int r = i / NQ, j = i - r * NQ;
      const uint8_t* row = g + reflect101(r0 + r - R, FH) * PITCH;
      uint32_t v = 0;
#pragma unroll
      for (int e = 0; e < 4; e++) {
        int x = 4 * j + e - R;
        x = x < 0 ? -x : x;
        x = x >= FW ? 2 * FW - 2 - x : x;
        x = min(max(x, 0), FW - 1);  // columns past W + R (never used) stay in the row
        v |= (uint32_t)row[x] << (8 * e);
      }
      *reinterpret_cast<uint32_t*>(&gface[r * C::GP + 4 * j]) = v;
    }
  };
  // this workgroup's rows [yb, ye): the whole face, or (SPLIT) its share of the face's bands
  int yb = 0, ye = FH, nwg = 1;
  if (SPLIT) {
    const int nbands = (FH + BY - 1) / BY, per = (nbands + gridDim.y - 1) / gridDim.y;
    nwg = (nbands + per - 1) / per;
    if ((int)blockIdx.y >= nwg) return;
    yb = blockIdx.y * per * BY;
    ye = min(FH, yb + per * BY);
  }
  // the padded rows of those bands, once: up to the last band's end (whole bands + 2R: every row the V
  // pass reads is staged)
  if (!TALL) stage_rows(yb, (ye - yb + BY - 1) / BY * BY + 2 * R);

#pragma unroll 1
  for (int y0 = yb; y0 < ye; y0 += BY) {  // probe 5: epilogue only
    __syncthreads();  // the face is staged; the previous H pass is done with vg / vq
    if (TALL) {       // (the previous V pass is done with gface: the barrier before the H pass)
      stage_rows(y0, BY + 2 * R);
      __syncthreads();
    }
    // ---- H pass (below): thread = (row hr, column group cq), outputs x = CPT cq + k
    constexpr int NCQ = 128 / CPT;
    const int hr = tid / NCQ, cq = tid % NCQ, y = y0 + hr, x0 = CPT * cq;
    f2 acc0[CPT], acc4[CPT], ac[3][CPT], be[3][CPT];  // mu 0, mu 4; per horizontal set p = 1..3: (A, C), (B, E)
    float dc[CPT];
#pragma unroll
    for (int k = 0; k < CPT; k++) {
      dc[k] = 0.f;
      acc0[k] = acc4[k] = f2{0.f, 0.f};
#pragma unroll
      for (int p = 0; p < 3; p++) ac[p][k] = be[p][k] = f2{0.f, 0.f};
    }
    const int rb = hr * C::VP + cq;
    // V value at padded column x0 + u + R: slot (u + R) % CPT, offset (u + R) / CPT
#define GS_IDX(u) (rb + (((u) + R) & (CPT - 1)) * C::QS + (((u) + R) >> C::LC))
    if constexpr (QS) {
    // ---- V pass over planes [QLO, QLO + QN) (+ Vg when G): vq slot q - QLO
    auto vpass = [&](auto qlo_c, auto qn_c, auto g_c) {
      constexpr int QLO = decltype(qlo_c)::value, QN = decltype(qn_c)::value;
      constexpr bool G = decltype(g_c)::value;
#pragma unroll 1
      for (int i = tid; i < BY * C::SC; i += GS_THREADS) {
        const int r = i / C::SC, cc = i - r * C::SC;
        if (cc >= NPC) continue;
        const uint8_t* col = &gface[((TALL ? 0 : y0 - yb) + r + R) * C::GP + cc];
        float vgv = 0.f;
        f2 vqv[QN];
#pragma unroll
        for (int q = 0; q < QN; q++) vqv[q] = f2{0.f, 0.f};
#pragma unroll
        for (int t = R; t >= 1; t--) {
          const float a = (float)col[t * C::GP], b = (float)col[-t * C::GP];
          const f2 sd = f2{a, a} + f2{b, -b};  // (S, D) = (a + b, a - b), exact
          const float* c = cv + 12 * t;
          if (G) vgv = fmaf(c[0], sd.x, vgv);
#pragma unroll
          for (int q = 0; q < QN; q++)
            vqv[q] = __builtin_elementwise_fma(f2{c[2 + 2 * (QLO + q)], c[3 + 2 * (QLO + q)]}, sd, vqv[q]);
        }
        const float p0 = (float)col[0];
        if (G) vgv = fmaf(cv[0], p0, vgv);
#pragma unroll
        for (int q = 0; q < QN; q++)
          vqv[q] = __builtin_elementwise_fma(f2{cv[2 + 2 * (QLO + q)], cv[3 + 2 * (QLO + q)]}, f2{p0, p0}, vqv[q]);
        const int qi = r * C::VP + (cc & 3) * C::QS + (cc >> 2);
        if (G) vg[qi] = vgv;
#pragma unroll
        for (int q = 0; q < QN; q++) vq[q][qi] = vqv[q];
      }
    };
    auto h_g = [&]() {  // Vg: DC term and mu 0
#pragma unroll
      for (int u = -R; u <= R + 3; u++) {
        const float v = vg[GS_IDX(u)];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int t = u - k;
          if (t < -R || t > R) continue;
          const float* h = chh + 16 * (t + R);
          dc[k] = fmaf(h[2], v, dc[k]);
          acc0[k] = __builtin_elementwise_fma(f2{h[0], h[1]}, f2{v, v}, acc0[k]);
        }
      }
    };
    auto h_mu4 = [&](int slot) {  // q = 4: mu 4
#pragma unroll
      for (int u = -R; u <= R + 3; u++) {
        const f2 v = vq[slot][GS_IDX(u)];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int t = u - k;
          if (t < -R || t > R) continue;
          const float* h = chh + 16 * (t + R);
          acc4[k] = __builtin_elementwise_fma(f2{h[2], h[3]}, v, acc4[k]);
        }
      }
    };
    auto h_p = [&](auto p_c, int slot) {  // q = p + 1: the four sums shared by mu and its mirror
      constexpr int P = decltype(p_c)::value;
#pragma unroll
      for (int u = -R; u <= R + 3; u++) {
        const f2 v = vq[slot][GS_IDX(u)], vs = f2{v.y, v.x};
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int t = u - k;
          if (t < -R || t > R) continue;
          const float* h = chh + 16 * (t + R) + 4 * (P + 1);
          ac[P][k] = __builtin_elementwise_fma(f2{h[0], h[1]}, v, ac[P][k]);
          be[P][k] = __builtin_elementwise_fma(f2{h[2], h[3]}, vs, be[P][k]);
        }
      }
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using BT = std::integral_constant<bool, true>;
    using BF = std::integral_constant<bool, false>;
      // two plane halves (V planes 1-2 + Vg, then 3-4): half the V-plane LDS, 3 workgroups per CU
      vpass(I0{}, I2{}, BT{});
      __syncthreads();
      h_g();
      h_p(I0{}, 0);
      h_p(I1{}, 1);
      __syncthreads();  // the H pass is done with vg / vq slots
      vpass(I2{}, I2{}, BF{});
      __syncthreads();
      h_p(I2{}, 0);
      h_mu4(1);
    } else {
    // ---- V pass
#pragma unroll 1
    for (int i = tid; i < BY * C::SC; i += GS_THREADS) {
      const int r = i / C::SC, cc = i - r * C::SC;
      if (cc >= NPC) continue;
      const uint8_t* col = &gface[((TALL ? 0 : y0 - yb) + r + R) * C::GP + cc];
      float vgv = 0.f;
      f2 vqv[4];
#pragma unroll
      for (int q = 0; q < 4; q++) vqv[q] = f2{0.f, 0.f};
#pragma unroll
      for (int t = R; t >= 1; t--) {
        const float a = (float)col[t * C::GP], b = (float)col[-t * C::GP];
        const f2 sd = f2{a, a} + f2{b, -b};  // (S, D) = (a + b, a - b), exact
        const float* c = cv + 12 * t;
        vgv = fmaf(c[0], sd.x, vgv);
#pragma unroll
        for (int q = 0; q < 4; q++) vqv[q] = __builtin_elementwise_fma(f2{c[2 + 2 * q], c[3 + 2 * q]}, sd, vqv[q]);
      }
      const float p0 = (float)col[0];
      vgv = fmaf(cv[0], p0, vgv);
#pragma unroll
      for (int q = 0; q < 4; q++) vqv[q] = __builtin_elementwise_fma(f2{cv[2 + 2 * q], cv[3 + 2 * q]}, f2{p0, p0}, vqv[q]);
      const int qi = r * C::VP + (cc & (CPT - 1)) * C::QS + (cc >> C::LC);
      vg[qi] = vgv;
#pragma unroll
      for (int q = 0; q < 4; q++) vq[q][qi] = vqv[q];
    }
    __syncthreads();  // V planes ready
    // Vg: DC term and mu 0
#pragma unroll
    for (int u = -R; u <= R + CPT - 1; u++) {
      const float v = vg[GS_IDX(u)];
#pragma unroll
      for (int k = 0; k < CPT; k++) {
        const int t = u - k;
        if (t < -R || t > R) continue;
        const float* h = chh + 16 * (t + R);
        dc[k] = fmaf(h[2], v, dc[k]);
        acc0[k] = __builtin_elementwise_fma(f2{h[0], h[1]}, f2{v, v}, acc0[k]);
      }
    }
    // q = 4: mu 4
#pragma unroll
    for (int u = -R; u <= R + CPT - 1; u++) {
      const f2 v = vq[3][GS_IDX(u)];
#pragma unroll
      for (int k = 0; k < CPT; k++) {
        const int t = u - k;
        if (t < -R || t > R) continue;
        const float* h = chh + 16 * (t + R);
        acc4[k] = __builtin_elementwise_fma(f2{h[2], h[3]}, v, acc4[k]);
      }
    }
    // q = p = 1, 2, 3: the four sums shared by mu and its mirror (mu 2 / 6, mu 3 / 5)
#pragma unroll
    for (int p = 0; p < 3; p++) {
#pragma unroll
      for (int u = -R; u <= R + CPT - 1; u++) {
        const f2 v = vq[p][GS_IDX(u)], vs = f2{v.y, v.x};
#pragma unroll
        for (int k = 0; k < CPT; k++) {
          const int t = u - k;
          if (t < -R || t > R) continue;
          const float* h = chh + 16 * (t + R) + 4 * (p + 1);
          ac[p][k] = __builtin_elementwise_fma(f2{h[0], h[1]}, v, ac[p][k]);
          be[p][k] = __builtin_elementwise_fma(f2{h[2], h[3]}, vs, be[p][k]);
        }
      }
    }
#undef GS_IDX
    }
    f2 acc[CPT][7];
#pragma unroll
    for (int k = 0; k < CPT; k++) {
      acc[k][0] = acc0[k];
      acc[k][4] = acc4[k];
      acc[k][1] = f2{ac[0][k].x - be[0][k].x, ac[0][k].y + be[0][k].y};
      acc[k][2] = f2{ac[1][k].x - be[1][k].x, ac[1][k].y + be[1][k].y};
      acc[k][6] = f2{ac[1][k].x + be[1][k].x, ac[1][k].y - be[1][k].y};
      acc[k][3] = f2{ac[2][k].x - be[2][k].x, ac[2][k].y + be[2][k].y};
      acc[k][5] = f2{ac[2][k].x + be[2][k].x, ac[2][k].y - be[2][k].y};
    }
#undef GS_IDX
    if (y < FH) {
#pragma unroll
      for (int o = 0; o < 7; o++) {
        float m4[CPT];
#pragma unroll
        for (int k = 0; k < CPT; k++) {
          const float re = fmaf(-cdc, dc[k], acc[k][o].x), im = acc[k][o].y;
          const float i2 = im * im, r2 = re * re;
          m4[k] = mag_of<EXACT, GS_FAST>(i2 + r2, tiny);
          minmax_update<GS_MASK>(mn[o], mx[o], m4[k], x0 + k < FW);
        }
        // columns >= W land in the row's pitch padding, never read
        float* mp = &mag[fd.mag_off + ((int64_t)(NU * 7 + o) * FH + y) * PITCH + x0];
        if constexpr (CPT == 4) *reinterpret_cast<float4*>(mp) = make_float4(m4[0], m4[1], m4[2], m4[3]);
        else *reinterpret_cast<float2*>(mp) = make_float2(m4[0], m4[1]);
      }
    }
  }
  if (SPLIT) {
    if (!split_finish<EXACT>(mn, mx, tiny, force, split_mm + ((int64_t)blockIdx.x * 5 + NU) * 16, nwg,
                             redo + blockIdx.x))
      return;
  } else {
    mag_flag<EXACT>(tiny, redo, force);
  }
  gabor_normalise_integrate<GS_THREADS / 64>(fd, NU, mn, mx, mag, chan);
}

// --------------------------------------------------------------- traversal --
// Integral channels are stored modulo 2^16 (u16).  A rectangle sum R = d - b - c + a of a u8
// plane is computed as the sum of its top (h>>1 rows) and bottom halves, each taken mod 2^16:
// a half covers at most 22 x 11 pixels, so its true sum is <= 255*242 = 61,710 < 2^16 and the
// modular value is exact; R (<= 123,420) is then exact in 32 bits.
// ImageSample::evalTest (ImageSample.cpp:48-63): p = (int)(R / (float)area) equals the integer
// quotient for R in [0, 255*484] (tests/test_numerics.py checks all pairs); computed as an rcp
// estimate plus one integer correction step.
__device__ __forceinline__ int idiv_small(int R, int area) {
  int q = (int)((float)R * __builtin_amdgcn_rcpf((float)area));
  const int r = R - (int)__umul24((unsigned)q, (unsigned)area);  // q, area < 2^24
  q += (r >= area) ? 1 : 0;
  q -= (r < 0) ? 1 : 0;
  return q;
}

// I: integral (mod 2^16) at the rectangle's top-left corner; ld: row pitch (elements).
template <class P>
__device__ __forceinline__ int rect_mean16(P I, int ld, int w, int h) {
  // all offsets < 2^24: 24-bit multiplies (full rate) instead of v_mul_lo_u32
  const int h1 = h >> 1, r1 = (int)__umul24((unsigned)h1, (unsigned)ld), r2 = (int)__umul24((unsigned)h, (unsigned)ld);
  const uint32_t a = I[0], b = I[w], c = I[r1], d = I[r1 + w];
  const uint32_t e = I[r2], f = I[r2 + w];
  const uint32_t top = (d - c - b + a) & 0xFFFFu, bot = (f - e - d + c) & 0xFFFFu;
  return idiv_small((int)(top + bot), (int)__umul24((unsigned)w, (unsigned)h));
}

// Node fields (ffd_device.hpp): rect offsets are encoded for PITCH; re-derive for a pitch `ld`.
__device__ __forceinline__ int node_off(uint32_t enc, int ld) {
  return (int)__umul24(enc >> 7, (unsigned)ld) + (int)(enc & 127u);
}

// ImageSample::evalTest's rectangle mean over the LDS window (k_traverse): p = byte address of the
// rectangle's top-left integral corner, ld2 = window row pitch in bytes.  The sum is taken as two
// halves split at h >> 1 rows, each exact modulo 2^16 (rect_mean16), and the quotient
// (int)(R / (float)(w*h)) as fma(R, rcp(area), 0.00075) truncated: equal to the integer quotient
// for every R in [0, 255 area], area in [1, 484], with rcp off by up to 2 ulp (tests/test_numerics.py).
// hh = h >> 1 (taken by the caller straight from the record's bits).
__device__ __forceinline__ int rect_mean_lds(const unsigned char* __restrict__ p, uint32_t w, uint32_t h, uint32_t hh,
                                             int ld2) {
  const int wb = (int)(2u * w);
  const int r1 = (int)__umul24(hh, (unsigned)ld2), r2 = (int)__umul24(h, (unsigned)ld2);
  const uint32_t area = __umul24(w, h);
  const uint32_t a = *reinterpret_cast<const uint16_t*>(p), b = *reinterpret_cast<const uint16_t*>(p + wb);
  const uint32_t f0 = *reinterpret_cast<const uint16_t*>(p + r2), f1 = *reinterpret_cast<const uint16_t*>(p + r2 + wb);
  const uint32_t c = *reinterpret_cast<const uint16_t*>(p + r1), d = *reinterpret_cast<const uint16_t*>(p + r1 + wb);
  // top = (a - b) + (d - c), bot = (f1 - f0) - (d - c), each mod 2^16, R = top + bot — in 32-bit registers, masked:
  // as u16 arithmetic the SLP vectorizer pairs a test's two rectangles into v_pk_sub_i16 / v_pk_add_u16 with
  // v_perm_b32 repacks and a v_pk_fma_f32 (round 6: FFD traversal 8.02-8.07 -> 7.94-7.99 ms)
  const uint32_t dc = d - c, top = (a - b + dc) & 0xFFFFu, bot = (f1 - f0 - dc) & 0xFFFFu;
  return (int)__builtin_fmaf((float)(top + bot), __builtin_amdgcn_rcpf((float)area), 0.00075f);
}

// Rectangle means of float-integral faces (FaceDesc::fint: the reference's CV_32F integral may round,
// FeatureChannelFactory.hpp:46-57 with OpenCV's float integral_): evalTest (ImageSample.cpp:48-63) on
// the rounded integral values, (int)((float)(d - b - c + a) / (float)area).  A rectangle half's mod-2^16
// combination is recovered in the window [-2048, 63488): its true value is the exact half sum (<= 61,710)
// plus the rounding errors of at most 11 row additions in each of two columns, each <= 64 (half an ulp)
// while the integrals stay below 2^31 (FINT_LIMIT, enforced by the host): |error| <= 1,408, so
// [-1,408, 63,118] lies inside the window.  Sums may then be negative or exceed 255 area, so the quotient
// is an IEEE division with truncation, as in the reference.
__device__ __forceinline__ int rect_mean_fint(const uint16_t* __restrict__ I, int ld, int w, int h) {
  const int h1 = h >> 1;
  const uint32_t a = I[0], b = I[w], c = I[h1 * ld], d = I[h1 * ld + w], e = I[h * ld], f = I[h * ld + w];
  auto half = [](uint32_t v) {
    v &= 0xFFFFu;
    return (int)v - (v >= 0xF800u ? 65536 : 0);  // [-2048, 63488)
  };
  const int R = half(d - c - b + a) + half(f - e - d + c);
  return (int)((float)R / (float)(w * h));
}

// Tree<S>::evaluateMT over global u16 planes (ffd_forest_eval_leaves hook); FINT: float-rounded integrals.
template <bool FINT = false>
__device__ __forceinline__ uint32_t walk16(const uint4* __restrict__ nodes, uint32_t node,
                                           const uint16_t* __restrict__ chan, int64_t plane) {
  uint4 nd = nodes[node];
  while (!(nd.x & LEAF_BIT)) {
    const uint16_t* I = chan + (int64_t)(nd.y & 63u) * plane;
    const uint16_t* I1 = I + node_off(nd.w & 0xFFFFu, PITCH);
    const uint16_t* I2 = I + node_off(nd.w >> 16, PITCH);
    const int p1 = FINT ? rect_mean_fint(I1, PITCH, (nd.y >> 6) & 31u, (nd.y >> 11) & 31u)
                        : rect_mean16(I1, PITCH, (nd.y >> 6) & 31u, (nd.y >> 11) & 31u);
    const int p2 = FINT ? rect_mean_fint(I2, PITCH, (nd.y >> 16) & 31u, (nd.y >> 21) & 31u)
                        : rect_mean16(I2, PITCH, (nd.y >> 16) & 31u, (nd.y >> 21) & 31u);
    node = nd.x + ((p1 - p2) <= (int)nd.z ? 0u : 1u);
    nd = nodes[node];
  }
  return nd.x & ~LEAF_BIT;
}

// Traversal of all (patch, tree) pairs of a batch.  Work unit = a G x G block of one face's patch
// grid with ALL the face's trees: the block's 38-channel u16 integral window (WW = 32 + step*(G-1)
// columns, WH = 32 + step_y*(G-1) rows) sits in LDS, so every rectangle read is an LDS read and only
// pair records come from L2.  The window fills the CU's LDS, so the kernel is persistent (one
// workgroup per CU) and software-pipelined: waves [NW/64, NT/64) load the NEXT block's window into
// registers while waves [0, NW/64) walk the current block; the registers are committed to LDS
// between blocks.  Blocks are dealt XCD-contiguously and face-major, so the 32 workgroups of an XCD
// share one or two faces' planes in that XCD's L2.
//
// A walk holds the 16-byte pair record of the node it stands on (both siblings' 56-bit tests,
// ffd_device.hpp "pair records"): the node's children pair is requested before its test is
// evaluated (one 16-byte load per visit), and the test picks the child.  The record gathers are what
// bounds the walk: one random 16-byte gather per lane costs the CU's vector-memory path about 2.4 cycles
// from L2 and 7.6 from the Infinity Cache (tools/td_probe.hip, profiles/r5a), and a block needs ~6,500 of
// them (500 walks x 13 deep levels).  Requesting both children's records a step ahead (two gathers per
// step) was measured even (round 5, DESIGN.md tried-table).
// Walker threads per workgroup by patch-block edge G: a block's G*G*T walks run in one round (T = 20
// FFD trees: 4x4 -> 320, 5x5 -> 500 of 512), the other threads stage the next window.  A block costs
// about its longest walk chain, so the walks a window holds per block set the throughput: FFD 5x5
// blocks with 512 walkers took the FFD pass from 10.4 to 8.6 ms at C2 (profiles/r2c).
constexpr int TRAV_NT = 1024;
__host__ __device__ constexpr int trav_nw(int GX, int GY, bool HP) { return GX * GY * (HP ? 15 : 20) <= 320 ? 320 : 512; }
// Window chunks held in registers per staging thread: 16-byte chunks when the window row pitch is
// a multiple of 8 columns, else 8-byte chunks (the pitch also sets the LDS bank pattern of the
// rectangle reads, so it is not padded up).
template <int CB, int NS> struct TravStage;
template <int NS> struct TravStage<8, NS> { static constexpr int U = (20480 + NS - 1) / NS; typedef uint32_t T __attribute__((ext_vector_type(2))); };
template <int NS> struct TravStage<16, NS> { static constexpr int U = (11000 + NS - 1) / NS; typedef uint32_t T __attribute__((ext_vector_type(4))); };
// Row-run staging (FFD 16-byte-chunk windows): NS threads over NCH x nq chunk columns, nh row groups per
// column, RU rows per group (the host checks RU <= TravStage::U, traverse_window_fits)
__host__ __device__ constexpr int trav_stage_groups(int ns, int nq) { return ns / (NCH * nq); }
__host__ __device__ constexpr int trav_stage_rows(int ns, int nq, int wh) {
  return trav_stage_groups(ns, nq) > 0 ? (wh + trav_stage_groups(ns, nq) - 1) / trav_stage_groups(ns, nq) : 1 << 20;
}

// LDS row pitch (u16) of a traversal window WW columns wide staged from a 4-element aligned column:
// a block starting at patch x px0 is staged from column px0 & ~3, so a block x-stride (gx * step)
// that is not a multiple of 4 needs up to 3 columns of slack.
__host__ __device__ __forceinline__ int trav_row_pitch(int WW, int xstride) {
  const int pad = (xstride & 3) ? 3 : 0;
  return (WW + pad + 3) & ~3;
}
__host__ __device__ __forceinline__ int trav_chunk_bytes(int WW, int xstride) { return trav_row_pitch(WW, xstride) % 8 == 0 ? 16 : 8; }

// Window bytes (16-byte aligned); the block's tree tops follow it (trav_top_n).
__host__ __device__ __forceinline__ int trav_window_bytes(int WW, int WH, int xstride) {
  return (NCH * WH * trav_row_pitch(WW, xstride) * 2 + 15) & ~15;
}

// Tree tops in LDS: for each of the block's T trees the first TOPN entries of its heap-ordered top
// table (TOP_CAP entries per tree in HBM, ffd_device.hpp "tree tops"): a 16-byte pair record and its
// global pair index each (20 B).  TOPN = the largest power of two <= top_max whose T tables fit in
// the LDS left over by the window (FFD 5x5 window, 20 trees: 8 entries = levels 0..2).
constexpr int TRAV_TOP_ENTRIES = 1400;  // tree-top entries a block stages at most (2 per staging thread)
__host__ __device__ __forceinline__ int trav_top_n(int T, int free_bytes, int top_max, int cap = TRAV_TOP_ENTRIES) {
  int n = TOP_CAP;
  while (n > 1 && (n > top_max || T * n * 20 > free_bytes || T * n > cap)) n >>= 1;
  return n;
}

constexpr int BUF_WORD3 = 0x00020000;  // raw buffer resource word 3 (gfx950: 32-bit data format)
#ifndef FFD_TRAV_TOUCH
#define FFD_TRAV_TOUCH 1  // k_traverse: touch the planes of the faces whose first block is this many iterations ahead (0: off)
#endif
#ifndef FFD_TRAV_TOUCH_SECT
#define FFD_TRAV_TOUCH_SECT 1  // words touched per 128-byte line (1: one; 2: one per 64-byte half)
#endif
#ifndef FFD_TRAV_TOUCH_HP
#define FFD_TRAV_TOUCH_HP 0  // 1: the head-pose pass touches too (4.34 -> 4.40 ms face-major, 4.48 with interleaved pairs)
#endif
#ifndef FFD_TRAV_ILV_HP
#define FFD_TRAV_ILV_HP 1  // head-pose faces dealt in interleaved groups of this many (2: 4.34 -> 4.44 ms without touches)
#endif
#ifndef FFD_TRAV_TOUCH_FIRST
#define FFD_TRAV_TOUCH_FIRST 0  // 1: the touches are issued before the next window's staging loads
#endif
#ifndef FFD_TRAV_PROBE_SAMEPLANES
#define FFD_TRAV_PROBE_SAMEPLANES 0
#endif
#ifndef FFD_TRAV_PROBE_WALKONLY
#define FFD_TRAV_PROBE_WALKONLY 0  // probe builds only: stage one window per workgroup, then walk without staging
#endif
#ifndef FFD_TRAV_STAGE_AUX
#define FFD_TRAV_STAGE_AUX 0  // cache-policy bits of the window staging loads (2: nt, 16: sc1 -- bypass the CU's L1)
#endif

constexpr int TRAV_BLK_BYTES = 64;  // the block descriptor the stagers hand to the walkers (end of the LDS)
struct TravArgs {
  const FaceDesc* faces;
  int n_faces, bpf;        // blocks per face: ceil(nx/G) * ceil(ny/G) (max over the batch)
  const uint4* pairs;      // pair records
  const uint4* tops;       // per tree: TOP_CAP heap-ordered pair records (levels 0..6)
  const uint32_t* top_idx; // ... and their global pair indices
  int top_free, top_max;   // LDS bytes after the window; cap on the entries staged per tree
  const uint32_t* far;     // per pair: offset of child 1's children pair when it exceeds 16 bits
  const HpState* hp_state; // FFD pass: selected trees; nullptr for the head-pose pass
  int ntrees_hp;           // head-pose pass: number of trees
  int step, step_y;        // patch grid steps (x, y)
  int plane;               // channel plane stride (elements), the same for every face of the batch
  int lds_bytes;           // dynamic LDS of the workgroup
  int tg;                  // tree groups per block (small batches: a block's trees over tg workgroups)
  const uint16_t* chan;
  int32_t* leaf_out;
};

template <bool HP, int GX, int GY, int CB, bool TGR = false>
__global__ __launch_bounds__(TRAV_NT) void k_traverse(TravArgs A) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint16_t* win = reinterpret_cast<uint16_t*>(smem);
  constexpr int NW = trav_nw(GX, GY, HP), NS = TRAV_NT - NW, U = TravStage<CB, NS>::U, GG = GX * GY;
  typedef typename TravStage<CB, NS>::T chunk_t;
  // tree-top entries a block stages at most: one per staging thread for the FFD 16-byte-chunk windows (the
  // 44 x 44 window leaves LDS for 8 levels-0..2 entries per tree; more registers would spill the stager role)
  constexpr int TOP_E = (!HP && CB == 16) ? NS : (TRAV_TOP_ENTRIES + NS - 1) / NS * NS;
  constexpr bool ROWS = !HP && CB == 16;  // row-run staging (below)
  const int tid = threadIdx.x;
  // window: WW integral columns x WH rows (steps may differ per axis: step_y, C4's (2, 1) grid)
  const int step = A.step, stepy = A.step_y, WW = 32 + step * (GX - 1), WH = 32 + stepy * (GY - 1);
  const int LW = trav_row_pitch(WW, GX * step), nq = LW * 2 / CB;
  const int total = NCH * WH * nq;  // chunks per window (host guarantees <= NS * U)
  uint4* top_rec = reinterpret_cast<uint4*>(smem + trav_window_bytes(WW, WH, GX * step));  // [t][TOPN] heap-ordered pairs
  // XCD-contiguous, face-major block range of this workgroup's XCD; workgroups of one XCD stride it
  // work unit lb = (face block, tree group): lb / tg = block, lb % tg = the group of the face's trees it walks
  const int tg = TGR ? A.tg : 1;  // TGR: the small-batch instance (tree groups); batches keep the plain indexing
  // ILV: the head-pose pass deals the blocks of two faces interleaved, so a face (30 blocks) spans two block
  // iterations of its XCD (32 workgroups) instead of one, and the plane touches of its first iteration (below) serve
  // its second
  constexpr int ILV = (HP && !TGR) ? FFD_TRAV_ILV_HP : 1;
  const int N = A.n_faces * A.bpf * tg, xcd = blockIdx.x & 7, k = blockIdx.x >> 3;
  const int q8 = N >> 3, r8 = N & 7;
  const int start = xcd * q8 + min(xcd, r8), end = start + q8 + (xcd < r8 ? 1 : 0);
  const int nk = gridDim.x >> 3;

  struct Blk {
    int f, xi0, yi0, px0, py0, nx, ny, T;
    int t0, t1;          // the trees of this work unit: [t0, t1) of the face's T
    int ok;
    int out_lo, out_hi;  // element offset of the face's leaf block (FaceDesc hp_off / mp_off)
    int more;            // 0: past the XCD's last block (every wave leaves its loop)
  };
  // The block a window holds, computed by the stagers with the window's next fill and handed to the walkers
  // through LDS at the end of the allocation (TRAV_BLK_BYTES), so the walkers start walking after the barrier
  // instead of loading the face descriptor and tree count themselves.
  static_assert(sizeof(Blk) <= TRAV_BLK_BYTES, "block descriptor slot");
  Blk* blk_lds = reinterpret_cast<Blk*>(smem + A.lds_bytes - TRAV_BLK_BYTES);
  auto block = [&](int lb) {
    Blk B;
    B.ok = 0;
    B.more = lb < end;
    const int lbb = TGR ? lb / tg : lb, g = TGR ? lb - lbb * tg : 0;
    int b;
    if constexpr (ILV > 1) {  // faces in groups of ILV, their blocks interleaved (the last group may be smaller)
      const int grp = lbb / (ILV * A.bpf), q = lbb - grp * (ILV * A.bpf), r = min(ILV, A.n_faces - grp * ILV);
      B.f = B.more ? grp * ILV + q % r : 0;
      b = B.more ? q / r : 0;
    } else {
      B.f = B.more ? lbb / A.bpf : 0;
      b = lbb - B.f * A.bpf;
    }
    const FaceDesc& fd = A.faces[B.f];
    B.nx = HP ? fd.nhx : fd.nmx;
    B.ny = HP ? fd.nhy : fd.nmy;
    const int gbx = max(1, (B.nx + GX - 1) / GX), gby = (B.ny + GY - 1) / GY;
    B.xi0 = (b % gbx) * GX;
    B.yi0 = (b / gbx) * GY;
    B.px0 = B.xi0 * step;
    B.py0 = B.yi0 * stepy;
    B.T = 0;
    if (B.more && fd.valid && !fd.fint && B.nx > 0 && b < gbx * gby) {  // (float-integral faces: k_walk_fint)
      B.ok = 1;
      B.T = HP ? A.ntrees_hp : A.hp_state[B.f].n_trees;
    }
    B.t0 = TGR ? g * B.T / tg : 0;
    B.t1 = TGR ? (g + 1) * B.T / tg : B.T;
    const int64_t off = HP ? fd.hp_off : fd.mp_off;
    B.out_lo = (int)(uint32_t)off;
    B.out_hi = (int)(off >> 32);
    return B;
  };

  auto walk_block = [&](const Blk& B) {
    const int items = GG * (TGR ? B.t1 - B.t0 : B.T), sh = B.px0 & 3;
    int32_t* out = A.leaf_out + (int64_t)(((uint64_t)(uint32_t)B.out_hi << 32) | (uint32_t)B.out_lo);
    const int ld2 = 2 * LW, chs2 = 2 * WH * LW;  // window row / channel-plane strides (bytes)
    const int topn = trav_top_n(B.T, A.top_free, A.top_max, TOP_E);
    const uint32_t* top_i = reinterpret_cast<const uint32_t*>(top_rec + B.T * topn);
    for (int item = tid; item < items; item += NW) {
      const int tr = item / GG, pl = item - tr * GG, t = TGR ? B.t0 + tr : tr;
      const int xi = B.xi0 + pl % GX, yi = B.yi0 + pl / GX;
      if (xi >= B.nx || yi >= B.ny) continue;
      // byte address of the patch's top-left integral corner in channel 0's window plane
      const unsigned char* base = reinterpret_cast<const unsigned char*>(win) +
                                  2 * ((yi - B.yi0) * stepy * LW + (xi - B.xi0) * step + sh);
      // (fields by bit-field extracts; bits of hi above 23 are the record's child offset, never read)
      auto test = [&](uint32_t lo, uint32_t hi) {
        const unsigned char* cb = base + __umul24(lo >> 26, (unsigned)chs2);
        const int p1 = rect_mean_lds(cb + __umul24(__builtin_amdgcn_ubfe(lo, 5, 5), (unsigned)ld2) + 2 * __builtin_amdgcn_ubfe(lo, 0, 5),
                                     __builtin_amdgcn_ubfe(hi, 0, 5), __builtin_amdgcn_ubfe(hi, 5, 5),
                                     __builtin_amdgcn_ubfe(hi, 6, 4), ld2);
        const int p2 = rect_mean_lds(cb + __umul24(__builtin_amdgcn_ubfe(lo, 15, 5), (unsigned)ld2) + 2 * __builtin_amdgcn_ubfe(lo, 10, 5),
                                     __builtin_amdgcn_ubfe(hi, 10, 5), __builtin_amdgcn_ubfe(hi, 15, 5),
                                     __builtin_amdgcn_ubfe(hi, 16, 4), ld2);
        // 10-bit two's complement: sign-extended thr[9:6] (hi[23:20]) above thr[5:0] (lo[25:20])
        const int thr = (int)(((uint32_t)__builtin_amdgcn_sbfe((int)hi, 20, 4) << 6) | __builtin_amdgcn_ubfe(lo, 20, 6));
        return (p1 - p2) <= thr ? 0u : 1u;  // Sample::eval: test <= threshold -> left (MPSample.cpp:77-84)
      };
      // levels 0..log2(topn): heap-ordered pair records in LDS (the children pair of node (h, s) is
      // entry 2h + s, of the root (h = 0) entry 1)
      const uint4* trec = top_rec + t * topn;
      uint32_t h = 0, s = 0;
      uint4 R = trec[0];
      uint32_t lo = R.x, hi = R.z;
      while (lo < (63u << 26)) {  // not a leaf (ch = 63)
        const uint32_t h2 = h ? 2u * h + s : 1u;
        if (h2 >= (uint32_t)topn) break;
        const uint4 Nr = trec[h2];
        s = test(lo, hi);
        h = h2;
        R = Nr;
        lo = s ? R.y : R.x;
        hi = s ? R.w : R.z;
      }
      // deeper levels: pair records from L2, the children pair requested before the test.  The children pair of
      // the current node is right after its own pair (child 0) or off1 away (child 1; off1 = 0: far[pair])
      uint32_t P = top_i[t * topn + h];
      while (lo < (63u << 26)) {  // not a leaf (ch = 63)
        const uint32_t off1 = (R.z >> 24) | ((R.w >> 24) << 8);
        uint32_t Q = P + (s ? off1 : 1u);
        if (s && off1 == 0u) Q = P + A.far[P];
        const uint4 Nr = A.pairs[Q];
        s = test(lo, hi);
        P = Q;
        R = Nr;
        lo = s ? R.y : R.x;
        hi = s ? R.w : R.z;
      }
      out[(xi * B.ny + yi) * B.T + t] = (int32_t)((lo & 0xFFFFFu) | hi << 20);  // reference order
    }
  };

  // Stager waves and walker waves run separate loops with the same barrier sequence per block
  // (waves are wholly one role), so the staging registers are live only in the stager loop and
  // the walkers get the rest of the register file.  Blocks of this workgroup: start + k, + nk, ...
  if (tid >= NW) {
    // Staging: chunk i = (channel c, window row r, 8-column group q), i = (c * WH + r) * nq + q, goes
    // to LDS chunk i; staging thread s owns chunks s + u * NS.  Their face-relative source byte
    // offsets c * plane + r * PITCH * 2 + q * 8 are the same for every block (every face of a batch has
    // the same plane stride, TravArgs::plane).
    chunk_t st[U];
    // tree tops of the next block (entry e = j + u * NS of its T x TOPN tables), reloaded only when
    // the face (and so the tree set) changes
    constexpr int TU = TOP_E / NS;
    typedef uint32_t rec_t __attribute__((ext_vector_type(4)));  // (a uint4 array lands in scratch)
    rec_t top_nd[TU];
    uint32_t top_p[TU];
    int top_face = -1;  // face whose tops the LDS holds after the next commit
    bool top_new = false;
    // Row runs (ROWS): staging thread s owns chunk column q of channel c over RU consecutive window rows
    // [g RU, g RU + RU) (g < nh row groups): its source offsets (rows PITCH * 2 bytes apart) and LDS
    // offsets (rows 2 LW bytes apart) are affine in the slot u, so both fold into instruction offsets
    // and no per-slot offset registers are held (the offset array spilled the FFD stager role: 80 B of
    // scratch per lane; FFD 8.91 -> 8.54 ms).  Used by the FFD 16-byte-chunk windows (5 x 5 at step 3); the
    // head-pose pass (no spill) keeps chunk i = s + u NS: row runs measured slower there (4.38 -> 4.62 ms).
    const int s0 = tid - NW, nh = trav_stage_groups(NS, nq), RU = trav_stage_rows(NS, nq, WH);
    const int sc = s0 / (nq * nh), sg = (s0 / nq) % nh, sq = s0 % nq;
    const int r_lo = sg * RU, r_n = sc < NCH ? max(0, min(RU, WH - r_lo)) : 0;  // this thread's rows
    // (chunk index form) chunk (c, r, q) of this thread's first chunk and the (c, r, q) step between its chunks
    const int dq = NS % nq, dr = (NS / nq) % WH, dc = NS / (nq * WH);
    const int q0 = s0 % nq, r0 = (s0 / nq) % WH, c0 = s0 / (nq * WH);
    int voffs[ROWS ? 1 : U];  // the U source offsets, precomputed once
    if constexpr (!ROWS) {
      int q = q0, r = r0, c = c0;
#pragma unroll
      for (int u = 0; u < U; u++) {
        voffs[u] = min(c, NCH) * A.plane * 2 + r * (PITCH * 2) + q * CB;
        q += dq;
        int cr = q >= nq;
        q -= cr ? nq : 0;
        r += dr + cr;
        cr = r >= WH;
        r -= cr ? WH : 0;
        c += dc + cr;
      }
    }
#if FFD_TRAV_PROBE_WALKONLY
    int staged = 0, committed = 0;
#endif
    auto prefetch = [&](const Blk& B) {
      if (!B.ok) return;
#if FFD_TRAV_PROBE_SAMEPLANES  // probe builds only: every block stages face 0's planes (always L2 / MALL-warm)
      const FaceDesc& fd = A.faces[0];
#else
      const FaceDesc& fd = A.faces[B.f];
#endif
      // the resource and the block offset must be wave-uniform (SGPRs): read them from the first lane
      const uint64_t base = (uint64_t)(A.chan + fd.ch_off);
      const uint32_t blo = __builtin_amdgcn_readfirstlane((uint32_t)base);
      const uint32_t bhi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
      const int nbytes = __builtin_amdgcn_readfirstlane((int)(NCH * fd.plane * 2));
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(((uint64_t)bhi << 32) | blo), (short)0, nbytes, BUF_WORD3);
      const int base_b = __builtin_amdgcn_readfirstlane((B.py0 * PITCH + (B.px0 & ~3)) * 2);
      // (reads past the face's planes return 0; chunks past the window are loaded but never committed)
      top_new = B.f != top_face;
      if (top_new) {
        top_face = B.f;
        const int topn = trav_top_n(B.T, A.top_free, A.top_max, TOP_E), lg = __builtin_ctz(topn);
#pragma unroll
        for (int u = 0; u < TU; u++) {
          const int e = tid - NW + u * NS;
          if (e < B.T * topn) {
            const int j = e >> lg, tree = HP ? j : A.hp_state[B.f].trees[j];
            const int g = tree * TOP_CAP + (e & (topn - 1));
            top_nd[u] = reinterpret_cast<const rec_t*>(A.tops)[g];
            top_p[u] = A.top_idx[g];
          }
        }
      }
#if FFD_TRAV_PROBE_WALKONLY  // probe: the window is staged once per workgroup (walks read a stale window)
      if (staged++) return;
#endif
      if constexpr (ROWS) {
        const int vb = min(sc, NCH - 1) * A.plane * 2 + r_lo * (PITCH * 2) + sq * CB;
#pragma unroll
        for (int u = 0; u < U; u++) {
          if (u < r_n) {
            if constexpr (CB == 16) st[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, vb + u * (PITCH * 2), base_b, FFD_TRAV_STAGE_AUX);
            else st[u] = __builtin_amdgcn_raw_buffer_load_b64(rs, vb + u * (PITCH * 2), base_b, FFD_TRAV_STAGE_AUX);
          }
        }
      } else {
#pragma unroll
        for (int u = 0; u < U; u++) {
          const int voff = voffs[u];
          if constexpr (CB == 16) st[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, base_b, FFD_TRAV_STAGE_AUX);
          else st[u] = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, base_b, FFD_TRAV_STAGE_AUX);
        }
      }
    };
    auto commit = [&](const Blk& B) {
      if (tid == NW) *blk_lds = B;  // the walkers' block (read after the barrier)
      if (!B.ok) return;
      chunk_t* dst = reinterpret_cast<chunk_t*>(win);
      const int s = tid - NW;
      if (top_new) {
        const int n = B.T * trav_top_n(B.T, A.top_free, A.top_max, TOP_E);
        uint32_t* top_i = reinterpret_cast<uint32_t*>(top_rec + n);
#pragma unroll
        for (int u = 0; u < TU; u++) {
          if (s + u * NS < n) {
            reinterpret_cast<rec_t*>(top_rec)[s + u * NS] = top_nd[u];
            top_i[s + u * NS] = top_p[u];
          }
        }
      }
#if FFD_TRAV_PROBE_WALKONLY
      if (committed++) return;
#endif
      if constexpr (ROWS) {
        unsigned char* db = smem + ((sc * WH + r_lo) * nq + sq) * CB;
#pragma unroll
        for (int u = 0; u < U; u++)
          if (u < r_n) *reinterpret_cast<chunk_t*>(db + u * (2 * LW)) = st[u];
      } else {
#pragma unroll
        for (int u = 0; u < U; u++)
          if (u * NS + s < total) dst[u * NS + s] = st[u];
      }
    };

    // Plane touches (FFD_TRAV_TOUCH): a face's planes are first read by its blocks' window staging (the channel kernels
    // wrote them long before, so they come from HBM), and every window of an iteration that overlaps a line in flight
    // waits for it.  So each block iteration the XCD's stager lanes load one word of every 128-byte line of the faces
    // whose first block the XCD reaches FFD_TRAV_TOUCH iterations later (the XCD's blocks are face-major), each line
    // once over the XCD's nk x NS lanes (<= 2 loads per lane per iteration); the words are consumed after the next
    // commit, whose wait for the staging loads covers them.  (Round-6 probes, DESIGN.md §5: the same lines fetched
    // through the scalar path with the stager waves waiting for them, or by a prefetching workgroup per XCD, were slower.)
    uint32_t pf_acc = 0, tv0 = 0, tv1 = 0;
    auto touch = [&](int it) {
      // (not in the 8-byte-chunk instances: C4's (2, 1) grid, whose stager registers already spill)
      if constexpr (FFD_TRAV_TOUCH > 0 && (FFD_TRAV_TOUCH_HP || !HP) && CB == 16) {
        const int b_lo = start + nk * (it + FFD_TRAV_TOUCH), b_hi = min(end, b_lo + nk), upf = A.bpf * tg * ILV;
        // only faces (groups of ILV faces) that take at most two block iterations: their lines all requested at once
        // then serve the next iteration; the blocks of a larger face (C4: 190 per face) come over many iterations,
        // by which time its touched lines are gone from L2 (C4 FFD 8.42 -> 9.83 ms touching them)
        if (b_lo >= b_hi || upf > 2 * nk) return;
        const int g_lo = (b_lo + upf - 1) / upf, g_hi = (b_hi + upf - 1) / upf;  // groups starting in the iteration
        const int f_lo = g_lo * ILV, f_hi = min(min(g_hi * ILV, A.n_faces), f_lo + 2);
        const int j = k * NS + (tid - NW);  // (the XCD has nk x NS stager lanes; lines past them are not touched)
        for (int f = f_lo; f < f_hi; f++) {
          const FaceDesc& fd = A.faces[f];
          if (!fd.valid || fd.fint || fd.nochan) continue;
          const int lpc = (fd.H + 1) * (PITCH * 2 / 128), T = NCH * lpc;  // 128-byte lines of the face's planes
          const uint32_t* base = reinterpret_cast<const uint32_t*>(A.chan + fd.ch_off);
          if (j < T) {
            const int c = j / lpc, o = j - c * lpc;
            uint32_t v = base[(int64_t)c * (A.plane / 2) + o * 32];
            if (FFD_TRAV_TOUCH_SECT > 1) v += base[(int64_t)c * (A.plane / 2) + o * 32 + 16];
            if (f == f_lo) tv0 = v; else tv1 = v;
          }
        }
      }
    };

    int lb = start + k;
    Blk cur = block(lb);
    prefetch(cur);
    for (int it = 0;; it++) {
      __syncthreads();  // the previous block's walks are done with the window
      commit(cur);
      __syncthreads();  // the window holds block `cur` (or the end marker)
      pf_acc += tv0 + tv1;  // (the last iteration's touches: complete, the commit waited for the loads before them)
      if (!cur.more) break;
      lb += nk;
      const Blk nxt = block(lb);
      if (FFD_TRAV_TOUCH_FIRST) touch(it);
      prefetch(nxt);
      if (!FFD_TRAV_TOUCH_FIRST) touch(it);
      cur = nxt;
    }
    if (pf_acc == 0x9E3779B9u && A.n_faces < 0) A.leaf_out[0] = (int32_t)pf_acc;  // (keeps the prefetch loads)
  } else {
    for (;;) {
      __syncthreads();
      __syncthreads();
      Blk cur = *blk_lds;
      if (!__builtin_amdgcn_readfirstlane(cur.more)) break;
      cur.ok = __builtin_amdgcn_readfirstlane(cur.ok);
      cur.T = __builtin_amdgcn_readfirstlane(cur.T);
      if (TGR) {
        cur.t0 = __builtin_amdgcn_readfirstlane(cur.t0);
        cur.t1 = __builtin_amdgcn_readfirstlane(cur.t1);
      }
      if (cur.ok) walk_block(cur);
    }
  }
}

// Forest<S>::evaluateMT over an explicit patch list (ffd_forest_eval_leaves hook).
__global__ void k_eval_patches(const uint4* __restrict__ nodes, const int32_t* __restrict__ roots,
                               const int32_t* __restrict__ tree_ids, int n_trees,
                               const int32_t* __restrict__ patches, int n_patches,
                               const uint16_t* __restrict__ chan, int64_t plane,
                               int32_t* __restrict__ leaf_ids, int fint) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_patches * n_trees) return;
  const int p = i / n_trees, t = i % n_trees;
  const uint16_t* I = chan + (int64_t)patches[2 * p + 1] * PITCH + patches[2 * p];
  const uint32_t root = (uint32_t)roots[tree_ids[t]];
  leaf_ids[i] = (int32_t)(fint ? walk16<true>(nodes, root, I, plane) : walk16(nodes, root, I, plane));
}

// Forest<S>::evaluateMT on patches of a device-resident ImageSample (ffd_sample_eval_leaves): one lane
// per (patch, tree) walk (Tree<S>::evaluateMT, Tree.hpp:173-191) over the 16-B nodes and the sample's u16
// planes.  Patches are either a list (inline in the argument block up to SAMPLE_INLINE, else `patches`) or
// a grid (x0 + xi step, y0 + yi step; patch p = xi * grid_ny + yi, the reference's x-major order).  The
// leaf ordinals go straight to leaf_out, which may be host-mapped pinned memory: a one-patch call is one
// launch and one stream synchronisation, no copies.
__global__ __launch_bounds__(256) void k_sample_eval(SampleEvalArgs A) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= A.n_patches * A.n_trees) return;
  const int p = i / A.n_trees, t = i - p * A.n_trees;
  int x, y;
  if (A.grid_ny > 0) {
    const int xi = p / A.grid_ny, yi = p - xi * A.grid_ny;
    x = A.x0 + xi * A.step;
    y = A.y0 + yi * A.step;
  } else if (A.n_patches <= SAMPLE_INLINE) {
    x = A.inl[2 * p];
    y = A.inl[2 * p + 1];
  } else {
    x = A.patches[2 * p];
    y = A.patches[2 * p + 1];
  }
  const uint16_t* I = A.chan + (int64_t)y * PITCH + x;
  const uint32_t root = (uint32_t)A.roots[A.trees[t]];
  A.leaf_out[i] = (int32_t)(A.fint ? walk16<true>(A.nodes, root, I, A.plane) : walk16(A.nodes, root, I, A.plane));
}

void launch_sample_eval(const SampleEvalArgs& a, hipStream_t s) {
  const int total = a.n_patches * a.n_trees;
  if (total <= 0) return;
  k_sample_eval<<<(total + 255) / 256, 256, 0, s>>>(a);
}

// The traversals of float-integral faces (FaceDesc::fint, rect_mean_fint above).  Grid (slices, faces);
// other faces exit at once.
template <bool HP>
__global__ __launch_bounds__(256) void k_walk_fint(const FaceDesc* __restrict__ faces, const uint4* __restrict__ nodes,
                                                  const int32_t* __restrict__ roots, int ntrees_hp,
                                                  const HpState* __restrict__ state, int step, int step_y,
                                                  const uint16_t* __restrict__ chan, int32_t* __restrict__ leaf_out) {
  const int f = blockIdx.y;
  const FaceDesc& fd = faces[f];
  if (!fd.valid || !fd.fint) return;
  const int nx = HP ? fd.nhx : fd.nmx, ny = HP ? fd.nhy : fd.nmy;
  const int T = HP ? ntrees_hp : state[f].n_trees;
  const int items = nx * ny * T;
  int32_t* out = leaf_out + (HP ? fd.hp_off : fd.mp_off);
  const uint16_t* base = chan + fd.ch_off;
  for (int it = blockIdx.x * 256 + threadIdx.x; it < items; it += gridDim.x * 256) {
    const int p = it / T, t = it - p * T;  // p = xi * ny + yi: the reference's patch order
    const int xi = p / ny, yi = p - xi * ny;
    const uint16_t* P = base + (yi * step_y) * PITCH + xi * step;
    uint32_t node = (uint32_t)roots[HP ? t : state[f].trees[t]];
    uint4 nd = nodes[node];
    while (!(nd.x & LEAF_BIT)) {
      const uint16_t* I = P + (int64_t)(nd.y & 63u) * fd.plane;
      const int p1 = rect_mean_fint(I + node_off(nd.w & 0xFFFFu, PITCH), PITCH, (nd.y >> 6) & 31u, (nd.y >> 11) & 31u);
      const int p2 = rect_mean_fint(I + node_off(nd.w >> 16, PITCH), PITCH, (nd.y >> 16) & 31u, (nd.y >> 21) & 31u);
      node = nd.x + ((p1 - p2) <= (int)nd.z ? 0u : 1u);
      nd = nodes[node];
    }
    out[it] = (int32_t)(nd.x & ~LEAF_BIT);
  }
}

// Sequential float sum acc += tp[0] + ... + tp[n - 1] in index order (one lane; tp 16-byte aligned):
// ds_read_b128 of 4 values at a time, a group of G reads in flight ahead of the adds.
__device__ __forceinline__ float serial_sum(const float* __restrict__ tp, int n, float acc) {
  constexpr int G = 4;
  const float4* t4 = reinterpret_cast<const float4*>(tp);
  const int n4 = n >> 2;
  int j = 0;
  float4 a[G];
  if (n4 >= G) {
#pragma unroll
    for (int e = 0; e < G; e++) a[e] = t4[e];
  }
  for (; j + 2 * G <= n4; j += G) {
    float4 b[G];
#pragma unroll
    for (int e = 0; e < G; e++) b[e] = t4[j + G + e];
#pragma unroll
    for (int e = 0; e < G; e++) {
      acc += a[e].x;
      acc += a[e].y;
      acc += a[e].z;
      acc += a[e].w;
    }
#pragma unroll
    for (int e = 0; e < G; e++) a[e] = b[e];
  }
  if (j + G <= n4) {
#pragma unroll
    for (int e = 0; e < G; e++) {
      acc += a[e].x;
      acc += a[e].y;
      acc += a[e].z;
      acc += a[e].w;
    }
    j += G;
  }
  for (; j < n4; j++) {
    const float4 x = t4[j];
    acc += x.x;
    acc += x.y;
    acc += x.z;
    acc += x.w;
  }
  for (int q = n4 * 4; q < n; q++) acc += tp[q];
  return acc;
}

// -------------------------------------------------- head pose + tree choice --
// getHeadPoseVotesMT reduction (face_utils.cpp:218-241) + areaUnderCurve (face_utils.cpp:304-323)
// + tree selection (FaceForest.cpp:214-250).  A 256-thread workgroup per HP_FACES faces.  The
// running float sums (sum m, sum m*m) are sequential by definition (the reference adds in leaf order:
// patch-major x-outer, tree-minor), so lane p < HP_FACES of wave 0 adds face p's leaves in that order; the
// leaf values arrive through LDS in tiles of 64 leaves per face, gathered by all four waves (wave w:
// faces w, w + 4, ...; leaf values three tiles ahead, their ids four, so the serial adds wait on
// neither).  Filtered-out leaves add +0, which leaves a non-negative float sum unchanged; the count
// of passing leaves (exact integer) comes from one ballot per face and tile.  Then the five pose-bin
// integrals (fp64 left Riemann sums) run on five lanes per face and lane p selects the trees.
constexpr int HP_T = 64;

template <int HP_FACES>
__global__ __launch_bounds__(256) void k_hp_pose(const FaceDesc* __restrict__ faces, int n_faces,
                                                 const int32_t* __restrict__ hp_leaf, const float* __restrict__ hp_m,
                                                 int hp_trees, int n_forests, int ntrees_per_forest,
                                                 HpState* __restrict__ state, FaceOut* __restrict__ out) {
  constexpr int HP_LD = HP_FACES + 1, HP_FPW = HP_FACES / 4;
  static_assert(HP_FACES % 4 == 0 && HP_FACES * 8 <= 256, "faces per workgroup");
  __shared__ float tm[HP_T * HP_LD], tq[HP_T * HP_LD];  // [leaf][face]: m (0 if filtered), m * m (0)
  __shared__ int s_total[HP_FACES], s_tcnt[HP_FACES], s_valid[HP_FACES];
  __shared__ int64_t s_off[HP_FACES];
  __shared__ int s_max;
  __shared__ float s_mean[HP_FACES], s_var[HP_FACES], s_area[HP_FACES][8];
  const int f0 = blockIdx.x * HP_FACES, tid = threadIdx.x, wv = tid >> 6, j = tid & 63;
  if (tid == 0) s_max = 0;
  __syncthreads();
  if (tid < HP_FACES) {
    const int f = f0 + tid;
    int total = 0, valid = 0;
    int64_t off = 0;
    if (f < n_faces) {
      const FaceDesc& fd = faces[f];
      FaceOut& o = out[f];
      o.bbox[0] = fd.bx; o.bbox[1] = fd.by; o.bbox[2] = fd.bw; o.bbox[3] = fd.bh;
      if (fd.valid) {  // (no head-pose patch: total 0, the reference's 0 / 0 pose)
        total = fd.nhx * fd.nhy * hp_trees;
        off = fd.hp_off;
        valid = 1;
      } else {
        o.status = fd.reject; o.n_trees = 0; state[f].n_trees = 0;
      }
    }
    s_total[tid] = total;
    s_off[tid] = off;
    s_valid[tid] = valid;
    atomicMax(&s_max, total);
  }
  __syncthreads();
  const int maxt = s_max;
  // values HP_PF tiles ahead of the adds (a shift register), their ids one tile further ahead
  constexpr int HP_PF = 3;
  int ids[HP_FPW];
  float vals[HP_PF][HP_FPW];
  auto load_ids = [&](int k0) {
#pragma unroll
    for (int i = 0; i < HP_FPW; i++) {
      const int p = wv + 4 * i, k = k0 + j;
      ids[i] = k < s_total[p] ? hp_leaf[s_off[p] + k] : -1;
    }
  };
  auto gather = [&](float (&v)[HP_FPW]) {  // -1: filtered leaf or past the end
#pragma unroll
    for (int i = 0; i < HP_FPW; i++) v[i] = ids[i] >= 0 ? hp_m[ids[i]] : -1.f;
  };
  float sum = 0.f, sum_sq = 0.f;
  int count = 0;
#pragma unroll
  for (int d = 0; d < HP_PF; d++) {
    load_ids(d * HP_T);
    gather(vals[d]);
  }
  load_ids(HP_PF * HP_T);
  for (int k0 = 0; k0 < maxt; k0 += HP_T) {
    // terms of tile k0 and this tile's passing-leaf counts
#pragma unroll
    for (int i = 0; i < HP_FPW; i++) {
      const int p = wv + 4 * i;
      const bool in = vals[0][i] >= 0.f;
      const float m = in ? vals[0][i] : 0.f;
      tm[j * HP_LD + p] = m;
      tq[j * HP_LD + p] = in ? m * m : 0.f;
      const int c = __popcll(__ballot(in));
      if (j == 0) s_tcnt[p] = c;
    }
#pragma unroll
    for (int d = 0; d + 1 < HP_PF; d++)
#pragma unroll
      for (int i = 0; i < HP_FPW; i++) vals[d][i] = vals[d + 1][i];
    if (k0 + HP_PF * HP_T < maxt) {
      gather(vals[HP_PF - 1]);                      // values of tile k0 + HP_PF * 64
      load_ids(k0 + (HP_PF + 1) * HP_T);            // ids one tile further
    }
    __syncthreads();
    if (tid < HP_FACES) {  // serial phase, in leaf order
      const int lim = min(HP_T, s_total[tid] - k0);
      count += s_tcnt[tid];
      int q = 0;
      for (; q + 8 <= lim; q += 8) {  // LDS reads 8 ahead of their in-order adds
        float vm[8], vq[8];
#pragma unroll
        for (int e = 0; e < 8; e++) {
          vm[e] = tm[(q + e) * HP_LD + tid];
          vq[e] = tq[(q + e) * HP_LD + tid];
        }
#pragma unroll
        for (int e = 0; e < 8; e++) {
          sum += vm[e];
          sum_sq += vq[e];
        }
      }
      for (; q < lim; q++) {
        sum += tm[q * HP_LD + tid];
        sum_sq += tq[q * HP_LD + tid];
      }
    }
    __syncthreads();
  }
  if (tid < HP_FACES && s_valid[tid]) {
    const float cnt = (float)count;  // the reference's float count of +1s is exact below 2^24
    float mean = sum / cnt;
    float var = (sum_sq / cnt) - (mean * mean);
    mean -= 2;
    var *= 0.05f;  // NORM_HEADPOSE_VARIANCE_FACTOR
    s_mean[tid] = mean;
    s_var[tid] = var;
  }
  __syncthreads();
  // areaUnderCurve per pose bin: lane (face p, bin j) = tid / 8, tid % 8 (fp64 left Riemann sums)
  if (tid < HP_FACES * 8) {
    const int p = tid >> 3, bin = tid & 7;
    if (s_valid[p] && bin < n_forests && bin < 5) {
      const float poseT[6] = {-2.5f, -0.35f, -0.20f, 0.20f, 0.35f, 2.5f};
      const double dmean = (double)s_mean[p], dstd = __builtin_sqrt((double)s_var[p]);
      double acc = 0, step = 0.01, tt;
      for (double x = poseT[bin]; x < (double)poseT[bin + 1]; x += step) {
        tt = (x - dmean) / dstd;
        acc += ffd_exp(-0.5 * (tt * tt)) * step;
      }
      s_area[p][bin] = (float)(acc * 1.0 / (dstd * 2.5066282746310002));
    }
  }
  __syncthreads();
  if (tid < HP_FACES && s_valid[tid]) {
    const int f = f0 + tid;
    const float mean = s_mean[tid], var = s_var[tid];
    FaceOut& o = out[f];
    o.status = 0;
    o.headpose = mean;
    o.pose_variance = var;
    HpState& s = state[f];
    s.headpose = mean;
    s.variance = var;
    float max_area = 0;
    int dominant = 0;  // first strict maximum
    for (int jj = 0; jj < n_forests; jj++) {
      const float a = s_area[tid][jj];
      s.pose_freq[jj] = a;
      if (max_area < a) { max_area = a; dominant = jj; }
    }
    int nt_total = 0;
    for (int i = 0; i < n_forests; i++) {
      const float v = floorf(s.pose_freq[i] * (float)ntrees_per_forest);
      int k = (v > -2147483649.0f && v < 2147483648.0f) ? (int)v : (int)0x80000000;
      k = min(k, ntrees_per_forest);
      for (int jj = 0; jj < k && nt_total < MAX_TREES; jj++) s.trees[nt_total++] = i * ntrees_per_forest + jj;
    }
    for (int i = nt_total; i < ntrees_per_forest; i++) s.trees[nt_total++] = dominant * ntrees_per_forest + i;
    s.n_trees = nt_total;
    o.n_trees = nt_total;
  }
}

// The same reduction for one face per workgroup (small batches: single-face latency).  Waves 1..3
// gather the face's leaf values in tiles of 768 leaves (4 per thread, values one tile ahead) into LDS
// (component-major: m and m * m planes, double-buffered); lanes 0 and 1 of wave 0 add the two planes in
// leaf order (serial_sum) while the next tile is gathered.  The pose-bin integrals: lane b walks bin b's
// abscissae (x += step, sequential as the reference's loop), every thread evaluates the Gaussian terms,
// lane b adds them in order; lane 0 selects the trees.
__global__ __launch_bounds__(256) void k_hp_pose1(const FaceDesc* __restrict__ faces, int n_faces,
                                                  const int32_t* __restrict__ hp_leaf, const float* __restrict__ hp_m,
                                                  int hp_trees, int n_forests, int ntrees_per_forest,
                                                  HpState* __restrict__ state, FaceOut* __restrict__ out) {
  constexpr int NT = 192, U1 = 4, T1 = NT * U1, NX = 224;  // bins span <= 2.15 / 0.01 + 1 abscissae
  __shared__ __attribute__((aligned(16))) float tv[2][2][T1];
  __shared__ double s_x[5][NX], s_t[5][NX];
  __shared__ int s_nx[5], s_cnt[4];
  __shared__ float s_sum[2], s_area[8];
  const int f = blockIdx.x, tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, tt = tid - 64;
  const bool gather_thread = tid >= 64;
  if (f >= n_faces) return;
  const FaceDesc& fd = faces[f];
  FaceOut& o = out[f];
  if (tid == 0) { o.bbox[0] = fd.bx; o.bbox[1] = fd.by; o.bbox[2] = fd.bw; o.bbox[3] = fd.bh; }
  if (!fd.valid) {
    if (tid == 0) { o.status = fd.reject; o.n_trees = 0; state[f].n_trees = 0; }
    return;
  }
  const int total = fd.nhx * fd.nhy * hp_trees;
  const int32_t* ids = hp_leaf + fd.hp_off;
  float v[U1];
  int count = 0;
  auto gather = [&](int k0) {
    int id[U1];
#pragma unroll
    for (int u = 0; u < U1; u++) id[u] = k0 + tt + NT * u < total ? ids[k0 + tt + NT * u] : -1;
#pragma unroll
    for (int u = 0; u < U1; u++) v[u] = id[u] >= 0 ? hp_m[id[u]] : -1.f;  // -1: filtered leaf or past the end
  };
  auto put = [&](int buf) {
#pragma unroll
    for (int u = 0; u < U1; u++) {
      const bool in = v[u] >= 0.f;
      const float m = in ? v[u] : 0.f;  // filtered leaves add +0 (a non-negative float sum is unchanged)
      count += in ? 1 : 0;
      tv[buf][0][tt + NT * u] = m;
      tv[buf][1][tt + NT * u] = in ? m * m : 0.f;
    }
  };
  float acc = 0.f;
  int buf = 0;
  if (gather_thread && total > 0) {
    gather(0);
    put(0);
    if (T1 < total) gather(T1);
  }
  __syncthreads();
  for (int k0 = 0; k0 < total; k0 += T1, buf ^= 1) {
    if (gather_thread) {
      if (k0 + T1 < total) {
        put(buf ^ 1);
        if (k0 + 2 * T1 < total) gather(k0 + 2 * T1);
      }
    } else if (tid < 2) {  // plane tid (sum m, sum m * m) in leaf order
      acc = serial_sum(&tv[buf][tid][0], min(T1, total - k0), acc);
    }
    __syncthreads();
  }
#pragma unroll
  for (int sh = 32; sh >= 1; sh >>= 1) count += __shfl_xor(count, sh);
  if (lane == 0) s_cnt[wv] = count;
  if (tid < 2) s_sum[tid] = acc;
  __syncthreads();
  const float cnt = (float)(s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3]);  // exact below 2^24
  float mean = s_sum[0] / cnt;
  float var = (s_sum[1] / cnt) - (mean * mean);
  mean -= 2;
  var *= 0.05f;  // NORM_HEADPOSE_VARIANCE_FACTOR
  const double dmean = (double)mean, dstd = __builtin_sqrt((double)var);
  const float poseT[6] = {-2.5f, -0.35f, -0.20f, 0.20f, 0.35f, 2.5f};
  const int nb = min(n_forests, 5);
  const double step = 0.01;
  if (tid < nb) {  // the abscissae of bin tid, accumulated as the reference's loop does
    int m = 0;
    for (double x = poseT[tid]; x < (double)poseT[tid + 1] && m < NX; x += step) s_x[tid][m++] = x;
    s_nx[tid] = m;
  }
  __syncthreads();
  for (int b = 0; b < nb; b++)
    for (int k = tid; k < s_nx[b]; k += 256) {
      const double tt = (s_x[b][k] - dmean) / dstd;
      s_t[b][k] = ffd_exp(-0.5 * (tt * tt)) * step;
    }
  __syncthreads();
  if (tid < nb) {
    double a = 0;
    for (int k = 0; k < s_nx[tid]; k++) a += s_t[tid][k];
    s_area[tid] = (float)(a * 1.0 / (dstd * 2.5066282746310002));
  }
  __syncthreads();
  if (tid == 0) {
    o.status = 0;
    o.headpose = mean;
    o.pose_variance = var;
    HpState& st = state[f];
    st.headpose = mean;
    st.variance = var;
    float max_area = 0;
    int dominant = 0;  // first strict maximum
    for (int jj = 0; jj < n_forests; jj++) {
      const float a = s_area[jj];
      st.pose_freq[jj] = a;
      if (max_area < a) { max_area = a; dominant = jj; }
    }
    int nt_total = 0;
    for (int i = 0; i < n_forests; i++) {
      const float vv = floorf(st.pose_freq[i] * (float)ntrees_per_forest);
      int kk = (vv > -2147483649.0f && vv < 2147483648.0f) ? (int)vv : (int)0x80000000;
      kk = min(kk, ntrees_per_forest);
      for (int jj = 0; jj < kk && nt_total < MAX_TREES; jj++) st.trees[nt_total++] = i * ntrees_per_forest + jj;
    }
    for (int i = nt_total; i < ntrees_per_forest; i++) st.trees[nt_total++] = dominant * ntrees_per_forest + i;
    st.n_trees = nt_total;
    o.n_trees = nt_total;
  }
}

// ------------------------------------------------------------ vote lists ----
// getFacialFeaturesVotesMT vote filter (face_utils.cpp:276-301).  A wave walks the face's FFD leaves
// [beg, end) in reference order (patch-major x-outer, tree-minor), 64 at a time; for each landmark a
// ballot + popcount gives every voting lane its slot after cnt[i], so the compacted list keeps the
// reference's vote order exactly.
#ifndef FFD_VOTE_U
#define FFD_VOTE_U 2
#endif
// VT: Vote, or VoteW for a wide face (FaceDesc::wide: positions beyond int16)
template <bool compact, class VT>
__device__ __forceinline__ void votes_range(const FaceDesc& fd, const int32_t* __restrict__ L,
                                            const uint4* __restrict__ leaf_rec, int bias_x, int bias_y, int T,
                                            int step, int step_y, int half_patch, int beg, int end,
                                            VT* __restrict__ V, int64_t cap, int (&cnt)[NPARTS]) {
  const int lane = __lane_id();
  const int ny = fd.nmy;
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  constexpr int U = FFD_VOTE_U;  // 64-item batches whose loads are in flight together
  // software pipeline over groups of U batches: the leaf ids of group g + 2 and the leaf records of
  // group g + 1 are in flight while group g is filtered
  struct Grp {
    int leaf[U], vx0[U], vy0[U];
    uint4 r0[U], r1[U], r2[compact ? 1 : U];
  };
  auto load_ids = [&](int base, Grp& G) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int k = base + u * 64 + lane;
      G.leaf[u] = -1;
      G.vx0[u] = G.vy0[u] = 0;
      if (k < end) {
        const int pr = idiv_small(k, T), xi = idiv_small(pr, ny), yi = pr - xi * ny;
        G.leaf[u] = L[k];  // leaves are stored in the reference order
        G.vx0[u] = fd.vox + xi * step + half_patch;  // patch.x + 15 (face_utils.cpp:257-293)
        G.vy0[u] = fd.voy + yi * step_y + half_patch;
      }
    }
  };
  // packed leaf records (see launch_votes): compact 32 B = 2 x uint4, else 64 B = 3 used uint4
  auto load_recs = [&](Grp& G) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      G.r0[u] = G.r1[u] = make_uint4(0, 0, 0, 0);
      if constexpr (!compact) G.r2[u] = make_uint4(0, 0, 0, 0);
      if (G.leaf[u] >= 0) {
        const uint4* rec = leaf_rec + (int64_t)G.leaf[u] * (compact ? 2 : 4);
        G.r0[u] = rec[0];
        G.r1[u] = rec[1];
        if constexpr (!compact) G.r2[u] = rec[2];
      }
    }
  };
  Grp cur, nxt;
  load_ids(beg, cur);
  load_recs(cur);
  load_ids(beg + 64 * U, nxt);
  for (int base = beg; base < end; base += 64 * U) {
    Grp nn;
    const bool more = base + 64 * U < end;
    if (more) {
      load_recs(nxt);
      load_ids(base + 2 * 64 * U, nn);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {  // batches in list order: (patch x-major, tree), then part
      const uint32_t mk = cur.r0[u].x;
      const float w = __uint_as_float(cur.r0[u].y);
      uint32_t off[NPARTS];
      if constexpr (compact) {  // u8 pairs relative to the biases -> the 64-B format's x | y << 16
        const uint32_t pk[5] = {cur.r0[u].z, cur.r0[u].w, cur.r1[u].x, cur.r1[u].y, cur.r1[u].z};
#pragma unroll
        for (int i = 0; i < NPARTS; i++) {
          const uint32_t v = (pk[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
          off[i] = (uint32_t)(uint16_t)((int)(v & 0xFFu) + bias_x) | (uint32_t)(uint16_t)((int)(v >> 8) + bias_y) << 16;
        }
      } else {
        const uint32_t o[NPARTS] = {cur.r0[u].z, cur.r0[u].w, cur.r1[u].x, cur.r1[u].y, cur.r1[u].z,
                                    cur.r1[u].w, cur.r2[u].x, cur.r2[u].y, cur.r2[u].z, cur.r2[u].w};  // (!compact)
#pragma unroll
        for (int i = 0; i < NPARTS; i++) off[i] = o[i];
      }
#pragma unroll
      for (int i = 0; i < NPARTS; i++) {  // mask bits >= n_parts are never set (engine load)
        const bool vote = (mk >> i) & 1u;
        const uint64_t bal = __ballot(vote);
        if (vote) {
          const int pos = cnt[i] + __popcll(bal & below);
          const int32_t o = (int32_t)off[i];
          const int vx = (int)(int16_t)(o & 0xFFFF) + cur.vx0[u], vy = (int)(int16_t)(o >> 16) + cur.vy0[u];
          if constexpr (sizeof(VT) == sizeof(VoteW)) V[i * cap + pos] = VoteW{vx, vy, w, 0};
          else V[i * cap + pos] = Vote{(int16_t)vx, (int16_t)vy, w};
        }
        cnt[i] += __popcll(bal);
      }
    }
    if (!more) break;
    cur = nxt;
    nxt = nn;
  }
}

// One wave per face (large batches).
template <bool compact>
__global__ __launch_bounds__(256) void k_votes(const FaceDesc* __restrict__ faces, int n_faces,
                                               const int32_t* __restrict__ mp_leaf,
                                               const uint4* __restrict__ leaf_rec, int bias_x,
                                               int bias_y, const HpState* __restrict__ state,
                                               int tslots, int step, int step_y, int half_patch, int n_parts,
                                               Vote* __restrict__ votes, int32_t* __restrict__ vote_counts) {
  const int f = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (f >= n_faces) return;
  const FaceDesc& fd = faces[f];
  if (!fd.valid) return;
  const int n = fd.nmx * fd.nmy, T = state[f].n_trees;
  int cnt[NPARTS];
#pragma unroll
  for (int i = 0; i < NPARTS; i++) cnt[i] = 0;
  if (fd.wide)
    votes_range<compact>(fd, mp_leaf + fd.mp_off, leaf_rec, bias_x, bias_y, T, step, step_y, half_patch, 0, n * T,
                         reinterpret_cast<VoteW*>(votes + fd.vote_off), (int64_t)tslots * n, cnt);
  else
    votes_range<compact>(fd, mp_leaf + fd.mp_off, leaf_rec, bias_x, bias_y, T, step, step_y, half_patch, 0, n * T,
                         votes + fd.vote_off, (int64_t)tslots * n, cnt);
  if (lane < n_parts) {
    int c = 0;
#pragma unroll
    for (int i = 0; i < NPARTS; i++)
      if (i == lane) c = cnt[i];
    vote_counts[(int64_t)f * NPARTS + lane] = c;
  }
}

// A workgroup of 16 waves per face (small batches: single-face latency).  The face's leaf list is cut
// into 16 contiguous segments of whole 64-item batches; every wave first counts its segment's votes
// per landmark (the vote masks only), then, after a prefix over the waves, walks its segment again
// writing each vote at its final slot.  Same order, same lists as k_votes.
constexpr int VOTES_WG_WAVES = 16;
template <bool compact>
__global__ __launch_bounds__(64 * VOTES_WG_WAVES) void k_votes_wg(const FaceDesc* __restrict__ faces, int n_faces,
                                                                 const int32_t* __restrict__ mp_leaf,
                                                                 const uint4* __restrict__ leaf_rec, int bias_x,
                                                                 int bias_y, const HpState* __restrict__ state,
                                                                 int tslots, int step, int step_y, int half_patch,
                                                                 int n_parts, Vote* __restrict__ votes,
                                                                 int32_t* __restrict__ vote_counts) {
  __shared__ int s_cnt[VOTES_WG_WAVES][NPARTS];
  const int f = blockIdx.x, wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (f >= n_faces) return;
  const FaceDesc& fd = faces[f];
  if (!fd.valid) return;  // whole workgroup
  const int n = fd.nmx * fd.nmy, T = state[f].n_trees, total = n * T;
  const int seg = (total + 64 * VOTES_WG_WAVES - 1) / (64 * VOTES_WG_WAVES) * 64;
  const int beg = min(total, wv * seg), end = min(total, beg + seg);
  const int32_t* L = mp_leaf + fd.mp_off;
  // pass 1: this segment's votes per landmark (the masks, 4 batches in flight)
  int cnt[NPARTS];
#pragma unroll
  for (int i = 0; i < NPARTS; i++) cnt[i] = 0;
  for (int b0 = beg; b0 < end; b0 += 4 * 64) {
    uint32_t mk[4];
    int leaf[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int k = b0 + u * 64 + lane;
      leaf[u] = k < end ? L[k] : -1;
    }
#pragma unroll
    for (int u = 0; u < 4; u++) mk[u] = leaf[u] >= 0 ? leaf_rec[(int64_t)leaf[u] * (compact ? 2 : 4)].x : 0u;
#pragma unroll
    for (int u = 0; u < 4; u++)
#pragma unroll
      for (int i = 0; i < NPARTS; i++) cnt[i] += __popcll(__ballot((mk[u] >> i) & 1u));
  }
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < NPARTS; i++) s_cnt[wv][i] = cnt[i];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NPARTS; i++) {
    int b = 0;
    for (int w = 0; w < wv; w++) b += s_cnt[w][i];
    cnt[i] = b;
  }
  // pass 2: the votes at their final slots
  if (fd.wide)
    votes_range<compact>(fd, L, leaf_rec, bias_x, bias_y, T, step, step_y, half_patch, beg, end,
                         reinterpret_cast<VoteW*>(votes + fd.vote_off), (int64_t)tslots * n, cnt);
  else
    votes_range<compact>(fd, L, leaf_rec, bias_x, bias_y, T, step, step_y, half_patch, beg, end, votes + fd.vote_off,
                         (int64_t)tslots * n, cnt);
  if (wv == VOTES_WG_WAVES - 1 && lane < n_parts) {
    int c = 0;
#pragma unroll
    for (int i = 0; i < NPARTS; i++)
      if (i == lane) c = cnt[i];
    vote_counts[(int64_t)f * NPARTS + lane] = c;
  }
}

// -------------------------------------------------------------- MeanShift ----
// MeanShift::shift (MeanShift.hpp:41-135) for one landmark of MS_FACES faces per workgroup, then the
// rescale of FaceForest.cpp:255-257.  Each pass walks the vote lists in tiles of MS_TILE votes:
//   parallel phase: all 256 threads compute the per-vote terms (x*w, y*w, w) — element-wise ops
//                   with the reference's rounding — into LDS;
//   serial phase:   lane p (one per face) adds its face's MS_TILE terms in list order,
// so every running sum equals the reference's sequential float sum bit for bit.
#ifndef FFD_MS_FACES
#define FFD_MS_FACES 20  // 4096 faces x 10 landmarks = 2048 workgroups = one round of 8 per CU
#endif
static_assert(3 * FFD_MS_FACES <= 64, "k_meanshift: lanes 3p..3p+2 of wave 0 add face p (SUM3), so every face must sit in wave 0");
#ifndef FFD_MS_TILE
#define FFD_MS_TILE 64
#endif
#ifndef FFD_MS_THREADS
#define FFD_MS_THREADS 256
#endif
constexpr int MS_FACES = FFD_MS_FACES, MS_TILE = FFD_MS_TILE, MS_LD = MS_FACES + 1, MS_THREADS = FFD_MS_THREADS;
static_assert(MS_TILE == 64 && MS_THREADS == 256, "k_meanshift maps a face's tile onto one of 4 waves");
constexpr int MS_FPW = (MS_FACES + 3) / 4;  // faces per wave
#ifndef FFD_MS_RA
#define FFD_MS_RA 4
#endif
constexpr int MS_RA = FFD_MS_RA;  // serial phase: LDS reads in flight ahead of the adds
// serial phase: lanes 3p, 3p + 1, 3p + 2 add face p's x / y / w terms (round 5: 1.93 -> 1.62 ms against one
// lane adding all three).  Terms as [component][vote][face], MS_LD words per vote, the planes MS_TSTRIDE apart
// (a plane is 64 x 21 words = 0 mod 64 banks, so the three lanes of a face read different banks).  (Rows per face
// read four terms at a time with ds_read_b128, as k_meanshift4 does, measured 1.63 -> 2.05 ms here.)
constexpr int MS_TSTRIDE = MS_TILE * MS_LD + MS_LD;
#ifndef FFD_MS_DEFAULT
#define FFD_MS_DEFAULT 0  // 0: chosen per batch (launch_meanshift); 1 k_meanshift, 4 k_meanshift4, 5 k_meanshift5
#endif
#ifndef FFD_MS_SORT
#define FFD_MS_SORT 1  // k_meanshift over chains sorted by list length (k_ms_order)
#endif
#ifndef FFD_MS_K
#define FFD_MS_K 2  // k_meanshift4: votes per lane per tile (C4 MeanShift: 1 8.52-8.56, 2 8.51-8.55, 4 8.68-8.71, 8 14.1 ms)
#endif
#ifndef FFD_VOTES_WG_MAX
#define FFD_VOTES_WG_MAX 64  // batches of up to 64 faces: k_votes_wg (16 waves per face)
#endif
#ifndef FFD_MS5_CHAINS
#define FFD_MS5_CHAINS 640  // batches of up to 64 faces: k_meanshift5 (a workgroup per chain)
#endif

// MeanShift::getWeightedMean's weight of one vote (MeanShift.hpp:122-124): d = cv::norm(mean - pos)
// (double sqrt, rounded to float), w = weight * expf(-d / lamda).  lam_y > 0: RN(1 / lamda) for the
// exact ffd_div_rcp quotient (lamda == 10 only, checked for every float in tests/test_numerics.py);
// the argument of the exponential is <= 0, where ffd_expf_nonpos == ffd_expf.
// ffd_expf_nonpos (include/ffd_numerics.h) with its Horner steps as three-address v_fma_f64: the
// compiler's accumulating v_fmac_f64 form needs a v_mov_b64 copy of every register-held coefficient
// per step.  Same operations, same roundings (MeanShift 2.50 -> 2.41 ms at C2).
__device__ __forceinline__ double fma3_f64(double a, double b, double c) {
  double d;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
__device__ __forceinline__ float ms_expf_nonpos(float xf) {
  const int under = xf < -104.0f;
  const double x = (double)(under ? -104.0f : xf);
  int k;
  const double r = ffd_exp_reduce(x, &k);
  double p = 1.0 / 39916800.0;
  p = fma3_f64(p, r, 1.0 / 3628800.0);
  p = fma3_f64(p, r, 1.0 / 362880.0);
  p = fma3_f64(p, r, 1.0 / 40320.0);
  p = fma3_f64(p, r, 1.0 / 5040.0);
  p = fma3_f64(p, r, 1.0 / 720.0);
  p = fma3_f64(p, r, 1.0 / 120.0);
  p = fma3_f64(p, r, 1.0 / 24.0);
  p = fma3_f64(p, r, 1.0 / 6.0);
  p = __builtin_fma(p, r, 0.5);
  p = __builtin_fma(p, r, 1.0);
  p = __builtin_fma(p, r, 1.0);
  const float e = (float)__builtin_ldexp(p, k);
  return under ? 0.0f : e;
}

// sqrt of s = dx^2 + dy^2 (binary32 dx, dy): the compiler's correctly rounded binary64 sequence (rsq, then the
// Goldschmidt / Newton steps, in its order) without its input scaling, which applies only below 2^-767 — such an
// s is 0 or at least 2^-298 — and with s = 0 selected through (the +inf case is unreachable).  Used by k_meanshift
// (C2 MeanShift 1.60 -> 1.53 ms); k_meanshift4 keeps the compiler's form (C4 7.54 with it, 7.84 ms without:
// register allocation).
template <bool UNSCALED>
__device__ __forceinline__ double ms_sqrt_sum2(double s) {
  if (!UNSCALED) return __builtin_sqrt(s);
  const double y0 = __builtin_amdgcn_rsq(s);
  double g = s * y0, h = y0 * 0.5;
  const double r = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, r, g);
  h = __builtin_fma(h, r, h);
  double d = __builtin_fma(-g, g, s);
  g = __builtin_fma(d, h, g);
  d = __builtin_fma(-g, g, s);
  g = __builtin_fma(d, h, g);
  return s == 0.0 ? s : g;
}
template <bool UNSCALED = false>
__device__ __forceinline__ float ms_weight(float mx, float my, float x, float y, float w, float lamda, float lam_y) {
  const float dx = mx - x, dy = my - y;
  const float d = (float)ms_sqrt_sum2<UNSCALED>((double)dx * dx + (double)dy * dy);
  // (ffd_div_rcp_fast: no divergent branch for tiny d, the same weight bits; round 5: C2 MeanShift 1.62 -> 1.59,
  // C4 7.60 -> 7.47 ms)
  const float q = lam_y > 0.f ? ffd_div_rcp_fast(-d, lamda, lam_y) : -d / lamda;
  return w * ms_expf_nonpos(q);
}

// 8 waves per SIMD (<= 64 VGPRs): 8 workgroups per CU, so C2's 2048 workgroups run as one round
// The MS_FACES chains (face, landmark) of a workgroup run their passes and tiles in lockstep, so a
// workgroup costs about its LONGEST list times its slowest chain's passes.  order (k_ms_order): the
// chains sorted by list length, longest first, dealt MS_FACES per workgroup — similar lengths share a
// workgroup and the longest start first.  Without it: workgroup (x, y) = faces [20x, 20x + 20), landmark y.
// A chain's arithmetic does not depend on its slot, so the order changes no result.
__global__ __launch_bounds__(MS_THREADS) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_meanshift(const FaceDesc* __restrict__ faces, int n_faces,
                                                   int tslots, int n_parts, float lamda, float lam_y, int max_iter,
                                                   float stop, const Vote* __restrict__ votes,
                                                   const int32_t* __restrict__ vote_counts,
                                                   float* __restrict__ ms_mean, FaceOut* __restrict__ out,
                                                   const int32_t* __restrict__ order) {
  constexpr int PLANE = MS_TSTRIDE;
  __shared__ float tt[3 * PLANE];
  float* const tx = tt;
  float* const ty = tt + PLANE;
  float* const tw = tt + 2 * PLANE;
  __shared__ float s_mx[MS_FACES], s_my[MS_FACES];
  __shared__ int s_cnt[MS_FACES], s_live[MS_FACES], s_chain[MS_FACES];
  __shared__ int64_t s_vb[MS_FACES];
  __shared__ int s_maxcnt, s_nlive;
  const int tid = threadIdx.x;
  if (tid == 0) { s_maxcnt = 0; s_nlive = 0; }
  __syncthreads();
  if (tid < MS_FACES) {
    const int64_t n_chains = (int64_t)n_faces * NPARTS;
    int64_t chain;
    if (order) {
      const int64_t k = (int64_t)blockIdx.x * MS_FACES + tid;
      chain = k < n_chains ? order[k] : n_chains;
    } else {
      chain = (int64_t)(blockIdx.x * MS_FACES + tid) * NPARTS + blockIdx.y;
      if (blockIdx.x * MS_FACES + tid >= n_faces) chain = n_chains;
    }
    s_chain[tid] = (int)chain;
    const int f = chain < n_chains ? (int)(chain / NPARTS) : n_faces, part = (int)(chain % NPARTS);
    int cnt = 0;
    int64_t vb = 0;
    if (f < n_faces && faces[f].valid && !faces[f].wide) {  // (wide faces: k_meanshift5)
      const FaceDesc& fd = faces[f];
      cnt = vote_counts[(int64_t)f * NPARTS + part];
      vb = fd.vote_off + (int64_t)part * tslots * fd.nmx * fd.nmy;
      if (part >= n_parts) cnt = 0;
    }
    s_cnt[tid] = cnt;
    s_vb[tid] = vb;
    s_live[tid] = (f < n_faces && faces[f].valid && !faces[f].wide) ? 1 : 0;
    s_mx[tid] = 0.f;
    s_my[tid] = 0.f;
    atomicMax(&s_maxcnt, cnt);
  }
  __syncthreads();
  const int maxcnt = s_maxcnt;
  // lane p of wave 0 owns chain s_chain[p]; its sums live in registers (SUM3: lanes 3p + e, component e)
  float ax = 0, ay = 0, aw = 0;
  float acc = 0;
  const int sp = tid / 3, se = tid - 3 * sp;  // SUM3: the face and component this lane adds
  // pass = -1: getMean (terms x*w, y*w, w); pass >= 0: getWeightedMean iteration
  for (int pass = -1; pass < max_iter; pass++) {
    if (pass >= 0) {
      if (tid == 0) s_nlive = 0;
      __syncthreads();
      if (tid < MS_FACES && s_live[tid]) atomicAdd(&s_nlive, 1);
      __syncthreads();
      if (s_nlive == 0) break;
    }
    ax = ay = aw = 0;
    acc = 0;
    // wave w owns faces w + 4 i (i < MS_FPW): a face's MS_TILE = 64 votes of a tile are one wave's lanes,
    // so its count, list base and mean are wave-uniform.  The votes of tile k0 are loaded into
    // registers during tile k0 - 64's serial phase (the first tile's here).
    const int wv = tid >> 6, j = tid & 63;
    Vote vv[MS_FPW];
    auto load_tile = [&](int k0) {
#pragma unroll
      for (int i = 0; i < MS_FPW; i++) {
        const int p = wv + 4 * i, k = k0 + j;
        if (p < MS_FACES && s_live[p] && k < s_cnt[p]) vv[i] = votes[s_vb[p] + k];
      }
    };
    load_tile(0);
    for (int k0 = 0; k0 < maxcnt; k0 += MS_TILE) {
      // parallel phase; faces that converged or whose list ended skip the tile (the serial phase
      // reads none of it)
#pragma unroll
      for (int i = 0; i < MS_FPW; i++) {
        const int p = wv + 4 * i;
        if (p >= MS_FACES || !s_live[p] || k0 + j >= s_cnt[p]) continue;
        const Vote v = vv[i];
        const float fx = (float)v.x, fy = (float)v.y;
        const float w = pass < 0 ? v.w : ms_weight<true>(s_mx[p], s_my[p], fx, fy, v.w, lamda, lam_y);
        const int at = j * MS_LD + p;
        tx[at] = fx * w;
        ty[at] = fy * w;
        tw[at] = w;
      }
      if (k0 + MS_TILE < maxcnt) load_tile(k0 + MS_TILE);  // in flight during the serial phase
      __syncthreads();
      if (tid < 3 * MS_FACES && s_live[sp]) {  // serial phase, in list order, a component per lane
        const int lim = min(MS_TILE, s_cnt[sp] - k0);
        const float* src = tt + se * PLANE + sp;
        int j = 0;
        for (; j + MS_RA <= lim; j += MS_RA) {  // LDS reads of MS_RA terms ahead of their in-order adds
          float v[MS_RA];
#pragma unroll
          for (int q = 0; q < MS_RA; q++) v[q] = src[(j + q) * MS_LD];
#pragma unroll
          for (int q = 0; q < MS_RA; q++) acc += v[q];
        }
        for (; j < lim; j++) acc += src[j * MS_LD];
      }
      __syncthreads();
    }
    // face tid's sums from lanes 3 tid .. 3 tid + 2 of wave 0
    ax = __shfl(acc, 3 * tid);
    ay = __shfl(acc, 3 * tid + 1);
    aw = __shfl(acc, 3 * tid + 2);
    if (tid < MS_FACES && s_live[tid]) {
      if (aw > 0) { ax /= aw; ay /= aw; }
      if (pass < 0) {
        s_mx[tid] = ax;
        s_my[tid] = ay;
      } else {
        const float ddx = ax - s_mx[tid], ddy = ay - s_my[tid];
        if (__builtin_sqrt((double)ddx * ddx + (double)ddy * ddy) < (double)stop) s_live[tid] = 0;  // converged
        s_mx[tid] = ax;
        s_my[tid] = ay;
      }
    }
    __syncthreads();
  }
  if (tid < MS_FACES) {
    const int chain = s_chain[tid];
    const int f = chain < n_faces * NPARTS ? chain / NPARTS : n_faces, part = chain % NPARTS;
    if (f < n_faces && faces[f].valid && !faces[f].wide) {
      const float mx = s_mx[tid], my = s_my[tid];
      if (part < n_parts) {
        ms_mean[((int64_t)f * NPARTS + part) * 2] = mx;
        ms_mean[((int64_t)f * NPARTS + part) * 2 + 1] = my;
      }
      const float inv = 1.0f / faces[f].scale;  // FaceForest.cpp:255-257
      out[f].points[part][0] = part < n_parts ? cv_round((float)cv_round(mx) * inv) : 0;
      out[f].points[part][1] = part < n_parts ? cv_round((float)cv_round(my) * inv) : 0;
    }
  }
}

// MeanShift, wave-independent form (FFD_MS_KERNEL=4, the default): each wave runs C chains (a chain =
// one (face, landmark) vote list) through MeanShift::shift (MeanShift.hpp:41-135) on its own — no
// workgroup barriers, so a wave's passes end when ITS chains converge and its tiles end at ITS longest
// list.  A tile is 64 / C votes of each chain:
//   terms  lane l computes the term (x*w, y*w, w) of vote l mod V of chain l / V (V = 64 / C) into the
//          wave's LDS tile,
//   sums   lane 3c + e (e = x, y, w) adds component e of chain c's V terms in list order,
// in program order within the wave (LDS operations of one wave complete in order).  Every running sum
// is the reference's sequential float sum bit for bit; the terms use ms_weight.
// The wave's terms as [component][chain][vote] rows (TVP words, an odd multiple of V, so the 64 term lanes of
// one store hit 64 banks), read four at a time with ds_read_b128 by the sum lanes (round 5: the serial phase
// issues TV adds + TV / 4 reads per tile instead of TV + TV; C4 MeanShift 8.40 -> 7.65 ms against [vote][chain]
// float4 terms).
#ifndef FFD_MS4_WAVES
#define FFD_MS4_WAVES 1  // k_meanshift4: minimum waves per SIMD the register allocation must allow (8: <= 64 VGPRs)
#endif
template <int C, int K>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FFD_MS4_WAVES)))
void k_meanshift4(const FaceDesc* __restrict__ faces, int n_faces, int tslots,
                                                   int n_parts, float lamda, float lam_y, int max_iter, float stop,
                                                   const Vote* __restrict__ votes, const int32_t* __restrict__ vote_counts,
                                                   float* __restrict__ ms_mean, FaceOut* __restrict__ out,
                                                   const int32_t* __restrict__ order) {
  constexpr int V = 64 / C, TV = V * K;  // term lanes per chain; votes per chain per tile
  static_assert(3 * C <= 64 && V * C == 64, "chains per wave");
  constexpr int TVP = K % 2 ? TV : TV + V;  // an odd multiple of V: c * TVP + tk is 64 distinct banks
  static_assert(TVP % 4 == 0, "16-B aligned rows");
  __shared__ __attribute__((aligned(16))) float term[4][3 * C * TVP];  // per wave: [component e][chain c][vote j]
  __shared__ float s_mean[4][C][2];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t n_chains = (int64_t)n_faces * NPARTS;
  const int64_t ch0 = ((int64_t)blockIdx.x * 4 + wv) * C;
  if (ch0 >= n_chains) return;  // whole waves; no workgroup barrier below
  // term lanes: chain tc = lane / V, vote offset tk = lane % V
  const int tc = lane / V, tk = lane - tc * V;
  // order (k_ms_order): chains sorted by list length, so a wave's C chains have similar lengths
  auto chain_of = [&](int c) -> int64_t {
    const int64_t k = ch0 + c;
    return order ? (k < n_chains ? (int64_t)order[k] : n_chains) : k;
  };
  auto chain_info = [&](int c, int& cnt, int64_t& vb, int& valid) {
    const int64_t g = chain_of(c);
    cnt = 0;
    vb = 0;
    valid = 0;
    if (g < n_chains) {
      const int f = (int)(g / NPARTS), part = (int)(g - (int64_t)f * NPARTS);
      const FaceDesc& fd = faces[f];
      if (fd.valid && !fd.wide) {  // (wide faces: k_meanshift5)
        valid = 1;
        cnt = part < n_parts ? vote_counts[(int64_t)f * NPARTS + part] : 0;
        vb = fd.vote_off + (int64_t)part * tslots * fd.nmx * fd.nmy;
      }
    }
  };
  int t_cnt, t_valid;
  int64_t t_vb;
  chain_info(tc, t_cnt, t_vb, t_valid);
  // sum lanes: chain sc = lane / 3, component se = lane % 3 (lanes >= 3C idle in the sums)
  const int sc = lane / 3, se = lane - 3 * sc;
  const bool sum_lane = lane < 3 * C;
  int s_cnt = 0, s_valid = 0;
  int64_t s_vb = 0;
  if (sum_lane) chain_info(sc, s_cnt, s_vb, s_valid);
  int live = t_valid;                    // the term lane's chain is live
  int s_live = s_valid;                  // the sum lane's chain is live
  float mx = 0.f, my = 0.f;              // term lane: its chain's current mean
  float smx = 0.f, smy = 0.f;            // sum lane: its chain's current mean
  const Vote* vp = votes + t_vb;
  for (int pass = -1; pass < max_iter; pass++) {
    if (__ballot(live) == 0ull) break;  // every chain of the wave converged
    int lim = live ? t_cnt : 0;
    int maxcnt = lim;
#pragma unroll
    for (int sh = 32; sh >= 1; sh >>= 1) maxcnt = max(maxcnt, __shfl_xor(maxcnt, sh));
    const int slim = s_live ? s_cnt : 0;
    float acc = 0.f;
    Vote v[K];
#pragma unroll
    for (int u = 0; u < K; u++) {
      v[u] = Vote{0, 0, 0.f};
      if (tk + V * u < lim) v[u] = vp[tk + V * u];
    }
    for (int k0 = 0; k0 < maxcnt; k0 += TV) {
#pragma unroll
      for (int u = 0; u < K; u++) {
        const int k = k0 + tk + V * u;
        float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
        if (k < lim) {
          const float fx = (float)v[u].x, fy = (float)v[u].y;
          const float w = pass < 0 ? v[u].w : ms_weight(mx, my, fx, fy, v[u].w, lamda, lam_y);
          t = make_float4(fx * w, fy * w, w, 0.f);
        }
        if (k + TV < lim) v[u] = vp[k + TV];  // the next tile's votes, in flight during the sums
        float* const row = &term[wv][tc * TVP + tk + V * u];
        row[0] = t.x;
        row[C * TVP] = t.y;
        row[2 * C * TVP] = t.z;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (sum_lane) {
        const int n = min(TV, slim - k0);
        const float* tp = &term[wv][(se * C + sc) * TVP];
        int j = 0;
        for (; j + 8 <= n; j += 8) {  // two 16-B reads ahead of their eight in-order adds
          const float4 a = *reinterpret_cast<const float4*>(tp + j);
          const float4 b = *reinterpret_cast<const float4*>(tp + j + 4);
          acc += a.x; acc += a.y; acc += a.z; acc += a.w;
          acc += b.x; acc += b.y; acc += b.z; acc += b.w;
        }
        if (j + 4 <= n) {
          const float4 a = *reinterpret_cast<const float4*>(tp + j);
          acc += a.x; acc += a.y; acc += a.z; acc += a.w;
          j += 4;
        }
        for (; j < n; j++) acc += tp[j];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    // chain sc's (x, y, w) sums sit on lanes 3sc, 3sc + 1, 3sc + 2
    const int b = 3 * sc;
    float ax = __shfl(acc, b), ay = __shfl(acc, b + 1), aw = __shfl(acc, b + 2);
    if (sum_lane && se == 0 && s_live) {
      if (aw > 0) { ax /= aw; ay /= aw; }
      if (pass >= 0) {
        const float ddx = ax - smx, ddy = ay - smy;
        if (__builtin_sqrt((double)ddx * ddx + (double)ddy * ddy) < (double)stop) s_live = 0;
      }
      smx = ax;
      smy = ay;
      s_mean[wv][sc][0] = ax;
      s_mean[wv][sc][1] = ay;
    }
    // liveness of every chain to its sum lanes (from lane 3c) and term lanes
    s_live = __shfl(s_live, b) ;
    smx = __shfl(smx, b);
    smy = __shfl(smy, b);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    live = __shfl(s_live, 3 * tc) && t_valid;
    mx = s_mean[wv][tc][0];
    my = s_mean[wv][tc][1];
  }
  if (sum_lane && se == 0 && s_valid) {
    const int64_t g = chain_of(sc);
    const int f = (int)(g / NPARTS), part = (int)(g - (int64_t)f * NPARTS);
    if (part < n_parts) {
      ms_mean[((int64_t)f * NPARTS + part) * 2] = smx;
      ms_mean[((int64_t)f * NPARTS + part) * 2 + 1] = smy;
    }
    const float inv = 1.0f / faces[f].scale;  // FaceForest.cpp:255-257
    out[f].points[part][0] = part < n_parts ? cv_round((float)cv_round(smx) * inv) : 0;
    out[f].points[part][1] = part < n_parts ? cv_round((float)cv_round(smy) * inv) : 0;
  }
}

// MeanShift, chain-per-workgroup form for small batches (single-face latency): one 256-thread
// workgroup runs ONE chain (a face's vote list for one landmark) through MeanShift::shift
// (MeanShift.hpp:41-135), in tiles of 192 U votes double-buffered in LDS (component-major: x*w, y*w, w
// planes): waves 1..3 compute tile k + 1's terms while lanes 0..2 of wave 0 add the three components of
// tile k in list order (serial_sum), one barrier per tile.  The sums are the reference's sequential
// float sums bit for bit; the terms use ms_weight.  A batch of a few faces has only 10 chains per face,
// so what bounds the pass is one chain's serial adds, not the term arithmetic.
// wide_only: the companion launch of a batch kernel, for the batch's wide faces (FaceDesc::wide, VoteW lists),
// which the batch kernels skip; this form reads either list format.
template <int U>
__global__ __launch_bounds__(256) void k_meanshift5(const FaceDesc* __restrict__ faces, int n_faces, int tslots,
                                                   int n_parts, float lamda, float lam_y, int max_iter, float stop,
                                                   const Vote* __restrict__ votes, const int32_t* __restrict__ vote_counts,
                                                   float* __restrict__ ms_mean, FaceOut* __restrict__ out,
                                                   int wide_only) {
  constexpr int NT = 192, T = NT * U;
  __shared__ __attribute__((aligned(16))) float tc[2][3][T];
  __shared__ float s_acc[3], s_m[2];
  __shared__ int s_live;
  const int tid = threadIdx.x, tt = tid - 64;
  const bool term_thread = tid >= 64;
  const int f = blockIdx.x / NPARTS, part = blockIdx.x - f * NPARTS;
  if (f >= n_faces || !faces[f].valid || (wide_only && !faces[f].wide)) return;  // whole workgroup
  const FaceDesc& fd = faces[f];
  const int cnt = part < n_parts ? vote_counts[(int64_t)f * NPARTS + part] : 0;
  const int64_t lb = (int64_t)part * tslots * fd.nmx * fd.nmy;
  const Vote* vp = votes + fd.vote_off + lb;
  const VoteW* vpw = reinterpret_cast<const VoteW*>(votes + fd.vote_off) + lb;
  const bool wide = fd.wide != 0;
  float mx = 0.f, my = 0.f;
  for (int pass = -1; pass < max_iter; pass++) {
    float vx[U], vy[U], vw[U];  // the vote positions as floats (exact: |position| < 2^24)
    auto load = [&](int k0) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int k = k0 + tt + NT * u;
        if (k < cnt) {
          if (wide) {
            const VoteW q = vpw[k];
            vx[u] = (float)q.x; vy[u] = (float)q.y; vw[u] = q.w;
          } else {
            const Vote q = vp[k];
            vx[u] = (float)q.x; vy[u] = (float)q.y; vw[u] = q.w;
          }
        }
      }
    };
    auto terms = [&](int buf, int k0) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int k = k0 + tt + NT * u;
        if (k < cnt) {
          const float fx = vx[u], fy = vy[u];
          const float w = pass < 0 ? vw[u] : ms_weight(mx, my, fx, fy, vw[u], lamda, lam_y);
          tc[buf][0][tt + NT * u] = fx * w;
          tc[buf][1][tt + NT * u] = fy * w;
          tc[buf][2][tt + NT * u] = w;
        }
      }
    };
    float acc = 0.f;
    int buf = 0;
    if (term_thread && cnt > 0) {
      load(0);
      terms(0, 0);
      if (T < cnt) load(T);
    }
    __syncthreads();
    for (int k0 = 0; k0 < cnt; k0 += T, buf ^= 1) {
      if (term_thread) {
        if (k0 + T < cnt) {
          terms(buf ^ 1, k0 + T);
          if (k0 + 2 * T < cnt) load(k0 + 2 * T);
        }
      } else if (tid < 3) {  // component tid of this tile's terms, in list order
        acc = serial_sum(&tc[buf][tid][0], min(T, cnt - k0), acc);
      }
      __syncthreads();
    }
    if (tid < 3) s_acc[tid] = acc;
    __syncthreads();
    if (tid == 0) {
      float ax = s_acc[0], ay = s_acc[1];
      const float aw = s_acc[2];
      if (aw > 0) { ax /= aw; ay /= aw; }
      int live = 1;
      if (pass >= 0) {
        const float ddx = ax - mx, ddy = ay - my;
        if (__builtin_sqrt((double)ddx * ddx + (double)ddy * ddy) < (double)stop) live = 0;  // converged
      }
      s_m[0] = ax;
      s_m[1] = ay;
      s_live = live;
    }
    __syncthreads();
    mx = s_m[0];
    my = s_m[1];
    if (!s_live) break;
  }
  if (tid == 0) {
    if (part < n_parts) {
      ms_mean[((int64_t)f * NPARTS + part) * 2] = mx;
      ms_mean[((int64_t)f * NPARTS + part) * 2 + 1] = my;
    }
    const float inv = 1.0f / fd.scale;  // FaceForest.cpp:255-257
    out[f].points[part][0] = part < n_parts ? cv_round((float)cv_round(mx) * inv) : 0;
    out[f].points[part][1] = part < n_parts ? cv_round((float)cv_round(my) * inv) : 0;
  }
}

// ------------------------------------------------------------------ launch --
#ifndef FFD_GRAY_STAGE_MAX
#define FFD_GRAY_STAGE_MAX 48 * 1024  // batches whose largest source box is at most this many pixels: k_gray_resize<true>
#endif
void launch_gray_resize(const FaceDesc* faces, int n, const uint8_t* images, uint8_t* gray, hipStream_t s, int max_src) {
  // small batches: a face's pixels spread over 8 workgroups (single-face latency)
  if (n <= FFD_GABOR_SPLIT_MAX || max_src <= 0 || max_src > FFD_GRAY_STAGE_MAX)
    k_gray_resize<false><<<dim3(n, n <= FFD_GABOR_SPLIT_MAX ? 8 : 1), 256, 0, s>>>(faces, images, gray, 0);
  else
    k_gray_resize<true><<<n, 256, (max_src + 15) / 16 * 16, s>>>(faces, images, gray, max_src);
}

// dynamic LDS of k_gabor_sep: the padded u8 face of the tallest face of the batch, its rows rounded up
// to whole GS_BY-row bands (the V pass of the last band reads up to row ceil(FH / GS_BY) * GS_BY + 2R - 1)
int gabor_face_lds(int R, int max_h) {
  return ((max_h + GS_BY - 1) / GS_BY * GS_BY + 2 * R) * ((PITCH + 2 * R + 3) / 4 * 4);
}

// the banded (SPLIT) Gabor instances for a batch of n faces of at most max_h rows
bool gabor_split(int n, int max_h) {
  static const int split_max = [] {
    const char* v = std::getenv("FFD_GABOR_SPLIT_MAX");
    return v ? std::atoi(v) : FFD_GABOR_SPLIT_MAX;
  }();
  return n <= split_max && max_h <= MAX_FACE_H;
}

void launch_gabor(int nu, const FaceDesc* faces, int n, int max_h, const uint8_t* gray, const float* coef, float* mag,
                  uint16_t* chan, int* redo, int force_exact, uint32_t* split_mm, hipStream_t s) {
  if (n <= 0) return;
  const float* c = coef + GABOR_OFFS[nu];
  // small batches: a face's bands / tiles spread over workgroups (split_mm: n x 5 zeroed 16-word slots)
  const bool split = split_mm && gabor_split(n, max_h);
  // the fast instance, then the exact one over the faces it flagged (an empty pass in practice)
  int* rd = redo + (int64_t)nu * n;  // one flag array per scale: the scales may run on fork streams
  for (int exact = 0; exact < 2; exact++) {
    if (split) {
      const int nbands = (max_h + GS_BY - 1) / GS_BY, nb = std::min(nbands, FFD_GABOR_SPLIT_WG);
      const int per = (nbands + nb - 1) / nb;
#define FFD_GABOR_SPLIT(WV, RV)                                                                                   \
  (exact ? k_gabor_sep<WV, true, false, true> : k_gabor_sep<WV, false, false, true>)<<<dim3(n, nb), GS_THREADS,     \
      (per * GS_BY + 2 * RV) * ((PITCH + 2 * RV + 3) / 4 * 4), s>>>(faces, gray, c, mag, chan, rd, force_exact, split_mm)
      switch (nu) {
        case 4: FFD_GABOR_SPLIT(25, 12); break;
        case 3: FFD_GABOR_SPLIT(19, 9); break;
        case 2: FFD_GABOR_SPLIT(13, 6); break;
        case 1: FFD_GABOR_SPLIT(9, 4); break;
        default: {
          const int tiles = ((PITCH - 3 + GB_TX - 1) / GB_TX) * ((max_h + GB_TY - 1) / GB_TY);
          (exact ? k_gabor7<true, true> : k_gabor7<false, true>)<<<dim3(n, tiles), GB_THREADS, 0, s>>>(
              faces, gray, reinterpret_cast<const float4*>(c), mag, chan, rd, force_exact, split_mm);
          break;
        }
      }
#undef FFD_GABOR_SPLIT
      continue;
    }
#define FFD_GABOR_LAUNCH(WV, RV)                                                                              \
  if ((FFD_GS_CPT2S_MASK >> nu) & 1)                                                                            \
    (exact ? k_gabor_sep<WV, true, false, false, 2, 4> : k_gabor_sep<WV, false, false, false, 2, 4>)<<<n,        \
        gs_threads(2, 4), gabor_face_lds(RV, std::min(max_h, MAX_FACE_H)), s>>>(faces, gray, c, mag, chan, rd,     \
                                                                                force_exact, nullptr);         \
  else if ((FFD_GS_CPT2_MASK >> nu) & 1)                                                                        \
    (exact ? k_gabor_sep<WV, true, false, false, 2> : k_gabor_sep<WV, false, false, false, 2>)<<<n, gs_threads(2), \
        gabor_face_lds(RV, std::min(max_h, MAX_FACE_H)), s>>>(faces, gray, c, mag, chan, rd, force_exact, nullptr); \
  else                                                                                                          \
    (exact ? k_gabor_sep<WV, true, false> : k_gabor_sep<WV, false, false>)<<<n, GS_THREADS, gabor_face_lds(RV, std::min(max_h, MAX_FACE_H)), s>>>(faces, gray, c, \
                                                                                                  mag, chan, rd, force_exact, nullptr); \
  if (max_h > MAX_FACE_H || FFD_GABOR_BAND_ALL)                                                                 \
    (exact ? k_gabor_sep<WV, true, true> : k_gabor_sep<WV, false, true>)<<<n, GS_THREADS, (GS_BY + 2 * RV) * ((PITCH + 2 * RV + 3) / 4 * 4), s>>>(faces, gray, c, \
                                                                                                  mag, chan, rd, force_exact, nullptr)
    switch (nu) {
      case 4: FFD_GABOR_LAUNCH(25, 12); break;
      case 3: FFD_GABOR_LAUNCH(19, 9); break;
      case 2: FFD_GABOR_LAUNCH(13, 6); break;
      case 1: FFD_GABOR_LAUNCH(9, 4); break;
      default:
        (exact ? k_gabor7<true, false> : k_gabor7<false, false>)<<<n, GB_THREADS, 0, s>>>(faces, gray, reinterpret_cast<const float4*>(c),
                                                                          mag, chan, rd, force_exact, nullptr);
        break;
    }
#undef FFD_GABOR_LAUNCH
  }
}

// Exhaustive device check of mag_sqrt against sqrtf (ffd_check_mag_sqrt): the n floats with bits
// [lo, lo + n); one mismatch count per wave (plain vector stores).
__global__ __launch_bounds__(256) void k_check_mag_sqrt(uint32_t lo, uint32_t n, uint32_t* __restrict__ bad) {
  uint32_t cnt = 0;
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
    const float s = __uint_as_float(lo + i);
    cnt += __float_as_uint(mag_sqrt(s)) != __float_as_uint(__builtin_sqrtf(s)) ? 1u : 0u;
  }
  for (int sh = 32; sh >= 1; sh >>= 1) cnt += (uint32_t)__shfl_xor((int)cnt, sh);
  if ((threadIdx.x & 63) == 0) bad[blockIdx.x * 4 + (threadIdx.x >> 6)] = cnt;
}

void launch_check_mag_sqrt(uint32_t lo, uint32_t n, uint32_t* bad, int blocks, hipStream_t s) {
  k_check_mag_sqrt<<<blocks, 256, 0, s>>>(lo, n, bad);
}

void launch_integral(const FaceDesc* faces, int n, int max_h, const uint8_t* gray, uint16_t* chan, hipStream_t s) {
  if (n <= 0) return;
  // the face's gray rows staged in LDS (<= 75 KB): small batches, and batches (FFD_INTEGRAL_STAGE_ALL: the byte reads
  // of the three scans at LDS rather than the texture path)
  if ((n <= FFD_GABOR_SPLIT_MAX || FFD_INTEGRAL_STAGE_ALL) && max_h <= MAX_FACE_H)
    k_integral<true><<<n, 256, (size_t)max_h * PITCH, s>>>(faces, gray, chan);
  else
    k_integral<false><<<n, 256, 0, s>>>(faces, gray, chan);
}

int traverse_lds_bytes(TravShape g, int step, int step_y) {
  const int WW = 32 + step * (g.gx - 1), WH = 32 + step_y * (g.gy - 1);
  return trav_window_bytes(WW, WH, g.gx * step) + MAX_TREES * 20 + TRAV_BLK_BYTES;  // window + the block's root pairs + its descriptor
}

bool traverse_window_fits(TravShape g, bool hp, int step, int step_y, int lds_cap) {
  const int WW = 32 + step * (g.gx - 1), WH = 32 + step_y * (g.gy - 1);
  const int cb = trav_chunk_bytes(WW, g.gx * step);
  const int ns = TRAV_NT - trav_nw(g.gx, g.gy, hp);
  const int u = cb == 16 ? (11000 + ns - 1) / ns : (20480 + ns - 1) / ns;  // TravStage<cb, ns>::U
  if (!hp && cb == 16 && trav_stage_rows(ns, trav_row_pitch(WW, g.gx * step) * 2 / cb, WH) > u)
    return false;
  return traverse_lds_bytes(g, step, step_y) <= lds_cap && NCH * WH * (trav_row_pitch(WW, g.gx * step) * 2 / cb) <= ns * u;
}

// The block shapes instantiated (x x y patches): head pose 4x4, 5x4, 3x3; FFD 5x5, 4x4, 3x3 (measurement builds
// add others through FFD_TRAV_EXTRA_SHAPES, e.g. -DFFD_TRAV_EXTRA_SHAPES(X)=X(true,4,5)).
#ifndef FFD_TRAV_EXTRA_SHAPES
#define FFD_TRAV_EXTRA_SHAPES(X)
#endif
// (FFD 4x6, 480 walks with an unpadded pitch-44 window, measured 14.5 ms against 8.5 ms for 5x5.)
#define FFD_TRAV_SHAPES(X)                                                                              \
  X(true, 4, 4) X(true, 5, 4) X(true, 3, 3) X(false, 5, 5) X(false, 4, 4) X(false, 3, 3) FFD_TRAV_EXTRA_SHAPES(X)

bool traverse_shape_supported(TravShape g, bool hp) {
#define FFD_TRAV_SUP(HPV, GXV, GYV) if (hp == HPV && g.gx == GXV && g.gy == GYV) return true;
  FFD_TRAV_SHAPES(FFD_TRAV_SUP)
#undef FFD_TRAV_SUP
  return false;
}


void launch_traverse(bool hp, const FaceDesc* faces, int n, int bpf, TravShape g, const uint4* pairs, const uint4* tops,
                     const uint32_t* top_idx, int top_max, const uint32_t* far, const HpState* state, int ntrees_hp,
                     int step, int step_y, int64_t plane, const uint16_t* chan, int32_t* leaf_out, int n_wg,
                     int lds_cap, hipStream_t s) {
  const int total_blocks = n * bpf;
  if (total_blocks <= 0) return;
  // a batch of a few faces has fewer blocks than CUs: a block's trees are then walked by tg workgroups, tg trees
  // fewer per window (single-face latency: the sample grid of the per-patch evaluateMT pattern, analyzeFace)
  const int tg = total_blocks * 2 <= n_wg ? std::max(1, std::min(hp ? 8 : 4, n_wg / total_blocks)) : 1;
  // the window, then as many tree-top entries as the rest of the CU's LDS holds
  const int WW = 32 + step * (g.gx - 1), WH = 32 + step_y * (g.gy - 1), lds = lds_cap;
  TravArgs A{faces, n, bpf, pairs, tops, top_idx, lds - trav_window_bytes(WW, WH, g.gx * step) - TRAV_BLK_BYTES, top_max,
             far, state, ntrees_hp, step, step_y, (int)plane, lds, tg, chan, leaf_out};
  // one persistent workgroup per CU, but no more than the blocks need (a one-face call has ~50 blocks)
  const int grid = std::max(8, std::min(n_wg & ~7, (total_blocks * tg + 7) & ~7));
  const bool c16 = trav_chunk_bytes(WW, g.gx * step) == 16;
#define FFD_TRAV_LAUNCH(HPV, GXV, GYV)                                                    \
  if (hp == HPV && g.gx == GXV && g.gy == GYV) {                                          \
    if (tg > 1) {                                                                         \
      if (c16) k_traverse<HPV, GXV, GYV, 16, true><<<grid, TRAV_NT, lds, s>>>(A);         \
      else k_traverse<HPV, GXV, GYV, 8, true><<<grid, TRAV_NT, lds, s>>>(A);              \
    } else if (c16) k_traverse<HPV, GXV, GYV, 16><<<grid, TRAV_NT, lds, s>>>(A);          \
    else k_traverse<HPV, GXV, GYV, 8><<<grid, TRAV_NT, lds, s>>>(A);                      \
    return;                                                                               \
  }
  FFD_TRAV_SHAPES(FFD_TRAV_LAUNCH)
#undef FFD_TRAV_LAUNCH
}

hipError_t set_gabor_lds_limit(int bytes) {
  hipError_t e = hipSuccess;
  const void* fns[] = {(const void*)k_gabor_sep<9, false, false>,  (const void*)k_gabor_sep<13, false, false>,
                       (const void*)k_gabor_sep<19, false, false>, (const void*)k_gabor_sep<25, false, false>,
                       (const void*)k_gabor_sep<9, true, false>,   (const void*)k_gabor_sep<13, true, false>,
                       (const void*)k_gabor_sep<19, true, false>,  (const void*)k_gabor_sep<25, true, false>,
                       (const void*)k_gabor_sep<13, false, false, false, 2>, (const void*)k_gabor_sep<19, false, false, false, 2>,
                       (const void*)k_gabor_sep<25, false, false, false, 2>, (const void*)k_gabor_sep<13, true, false, false, 2>,
                       (const void*)k_gabor_sep<19, true, false, false, 2>,  (const void*)k_gabor_sep<25, true, false, false, 2>,
                       (const void*)k_gabor_sep<9, false, false, false, 2, 4>, (const void*)k_gabor_sep<9, true, false, false, 2, 4>,
                       (const void*)k_gabor_sep<13, false, false, false, 2, 4>, (const void*)k_gabor_sep<19, false, false, false, 2, 4>,
                       (const void*)k_gabor_sep<25, false, false, false, 2, 4>, (const void*)k_gabor_sep<13, true, false, false, 2, 4>,
                       (const void*)k_gabor_sep<19, true, false, false, 2, 4>,  (const void*)k_gabor_sep<25, true, false, false, 2, 4>,
                       (const void*)k_integral<true>};
  for (const void* f : fns) {
    hipError_t r = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (r != hipSuccess) e = r;
  }
  return e;
}


hipError_t set_traverse_lds_limit(int bytes) {
  hipError_t e = hipSuccess;
#define FFD_TRAV_ATTR(HPV, GXV, GYV)                                                                     \
  for (const void* f : {(const void*)k_traverse<HPV, GXV, GYV, 8>, (const void*)k_traverse<HPV, GXV, GYV, 16>,        \
                        (const void*)k_traverse<HPV, GXV, GYV, 8, true>, (const void*)k_traverse<HPV, GXV, GYV, 16, true>}) { \
    hipError_t r = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);            \
    if (r != hipSuccess) e = r;                                                                          \
  }
  FFD_TRAV_SHAPES(FFD_TRAV_ATTR)
#undef FFD_TRAV_ATTR
  return e;
}

void launch_walk_fint(bool hp, const FaceDesc* faces, int n, const uint4* nodes, const int32_t* roots, int ntrees_hp,
                      const HpState* state, int step, int step_y, const uint16_t* chan, int32_t* leaf_out, hipStream_t s) {
  if (n <= 0) return;
  const dim3 grid(64, n);
  if (hp) k_walk_fint<true><<<grid, 256, 0, s>>>(faces, nodes, roots, ntrees_hp, state, step, step_y, chan, leaf_out);
  else k_walk_fint<false><<<grid, 256, 0, s>>>(faces, nodes, roots, ntrees_hp, state, step, step_y, chan, leaf_out);
}

void launch_eval_patches(const uint4* nodes, const int32_t* roots, const int32_t* tree_ids, int n_trees,
                         const int32_t* patches, int n_patches, const uint16_t* chan, int64_t plane,
                         int32_t* leaf_ids, hipStream_t s, bool fint) {
  const int total = n_patches * n_trees;
  if (total <= 0) return;
  k_eval_patches<<<(total + 255) / 256, 256, 0, s>>>(nodes, roots, tree_ids, n_trees, patches, n_patches, chan,
                                                     plane, leaf_ids, fint ? 1 : 0);
}

void launch_hp_pose(const FaceDesc* faces, int n, const int32_t* hp_leaf, const float* hp_m, int hp_trees,
                    int n_forests, int ntrees_per_forest, HpState* state, FaceOut* out, hipStream_t s) {
  static const int nf = [] {  // faces per workgroup (FFD_HP_FACES: 4, 8 or 16; C2: 0.261 / 0.256 / 0.281 ms)
    const char* v = std::getenv("FFD_HP_FACES");
    const int k = v ? std::atoi(v) : 8;
    return k == 4 || k == 16 ? k : 8;
  }();
  static const int one_max = [] {  // faces up to which a workgroup reduces each face (k_hp_pose1)
    const char* v = std::getenv("FFD_HP_ONE_MAX");
    return v ? std::atoi(v) : 64;
  }();
  if (n <= one_max) {
    k_hp_pose1<<<n, 256, 0, s>>>(faces, n, hp_leaf, hp_m, hp_trees, n_forests, ntrees_per_forest, state, out);
    return;
  }
  if (nf == 16)
    k_hp_pose<16><<<(n + 15) / 16, 256, 0, s>>>(faces, n, hp_leaf, hp_m, hp_trees, n_forests, ntrees_per_forest, state, out);
  else if (nf == 8)
    k_hp_pose<8><<<(n + 7) / 8, 256, 0, s>>>(faces, n, hp_leaf, hp_m, hp_trees, n_forests, ntrees_per_forest, state, out);
  else
    k_hp_pose<4><<<(n + 3) / 4, 256, 0, s>>>(faces, n, hp_leaf, hp_m, hp_trees, n_forests, ntrees_per_forest, state, out);
}

void launch_votes(const FaceDesc* faces, int n, const int32_t* mp_leaf, const uint4* leaf_rec, bool compact,
                  int bias_x, int bias_y, const HpState* state,
                  int tslots, int step, int step_y, int half_patch, int n_parts, Vote* votes, int32_t* vote_counts,
                  hipStream_t s) {
  static const int wg_max = [] {  // faces up to which a workgroup of 16 waves filters each face
    const char* v = std::getenv("FFD_VOTES_WG_MAX");
    return v ? std::atoi(v) : FFD_VOTES_WG_MAX;
  }();
  if (n <= wg_max) {
    if (compact)
      k_votes_wg<true><<<n, 64 * VOTES_WG_WAVES, 0, s>>>(faces, n, mp_leaf, leaf_rec, bias_x, bias_y, state, tslots, step,
                                                         step_y, half_patch, n_parts, votes, vote_counts);
    else
      k_votes_wg<false><<<n, 64 * VOTES_WG_WAVES, 0, s>>>(faces, n, mp_leaf, leaf_rec, bias_x, bias_y, state, tslots, step,
                                                          step_y, half_patch, n_parts, votes, vote_counts);
    return;
  }
  if (compact)
    k_votes<true><<<(n + 3) / 4, 256, 0, s>>>(faces, n, mp_leaf, leaf_rec, bias_x, bias_y, state, tslots, step, step_y,
                                              half_patch, n_parts, votes, vote_counts);
  else
    k_votes<false><<<(n + 3) / 4, 256, 0, s>>>(faces, n, mp_leaf, leaf_rec, bias_x, bias_y, state, tslots, step, step_y,
                                               half_patch, n_parts, votes, vote_counts);
}

// The chains (face, landmark) sorted by list length, longest first (counting sort on length / 32, one
// workgroup; the order within a bucket is the atomics' and changes no result).
constexpr int MS_ORDER_BUCKETS = 1024;
__global__ __launch_bounds__(1024) void k_ms_order(const FaceDesc* __restrict__ faces, int n_faces, int n_parts,
                                                   const int32_t* __restrict__ vote_counts, int32_t* __restrict__ order) {
  __shared__ int hist[MS_ORDER_BUCKETS];
  __shared__ int wsum[16];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int n_chains = n_faces * NPARTS;
  auto bucket = [&](int c) {  // descending length -> ascending bucket
    const int f = c / NPARTS, part = c - f * NPARTS;
    const int cnt = (part < n_parts && faces[f].valid) ? vote_counts[c] : 0;
    return MS_ORDER_BUCKETS - 1 - min(cnt >> 5, MS_ORDER_BUCKETS - 1);
  };
  hist[tid] = 0;
  __syncthreads();
  for (int c = tid; c < n_chains; c += 1024) atomicAdd(&hist[bucket(c)], 1);
  __syncthreads();
  const int v = hist[tid];
  int incl = v;
#pragma unroll
  for (int sh = 1; sh < 64; sh <<= 1) {
    const int t = __shfl_up(incl, sh);
    if (lane >= sh) incl += t;
  }
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  int base = 0;
  for (int w = 0; w < wv; w++) base += wsum[w];
  hist[tid] = base + incl - v;  // bucket start
  __syncthreads();
  for (int c = tid; c < n_chains; c += 1024) order[atomicAdd(&hist[bucket(c)], 1)] = c;
}

void launch_meanshift(const FaceDesc* faces, int n, const HpState* state, int tslots, int n_parts, float lamda,
                      int max_iter, float stop, const Vote* votes, const int32_t* vote_counts, float* ms_mean,
                      FaceOut* out, int32_t* order, hipStream_t s, bool any_wide) {
  (void)state;
  // k_meanshift5 (5) for a few chains (single-face latency: one workgroup per chain); k_meanshift (1) when
  // the batch has chains for >= 4 of its workgroups per CU (C2: 2,048 workgroups, 2.45 ms, where
  // k_meanshift4 takes 3.1 ms: its fp64 term chains run at lower occupancy); else the wave-independent
  // k_meanshift4 (4) (C4, 10,240 chains of ~30 k votes: 16.2 -> 9.4 ms)
  static const int forced = [] {
    const char* v = std::getenv("FFD_MS_KERNEL");
    return v ? std::atoi(v) : FFD_MS_DEFAULT;
  }();
  static const int64_t ms5_max = [] {  // chains up to which the chain-per-workgroup form runs
    const char* v = std::getenv("FFD_MS5_CHAINS");
    return v ? std::atoll(v) : (int64_t)FFD_MS5_CHAINS;
  }();
  const int64_t chains = (int64_t)n * NPARTS;
  const int which = forced ? forced : (chains <= ms5_max ? 5 : chains >= (int64_t)20 * 4 * 256 ? 1 : 4);
  const float lam_y = lamda == 10.f ? 1.f / 10.f : 0.f;  // the verified fast quotient (ffd_div_rcp)
  if (which == 5) {
    k_meanshift5<4><<<(unsigned)chains, 256, 0, s>>>(faces, n, tslots, n_parts, lamda, lam_y, max_iter, stop, votes,
                                                     vote_counts, ms_mean, out, 0);
    return;
  }
  if (any_wide)  // the batch kernels below skip wide faces
    k_meanshift5<4><<<(unsigned)chains, 256, 0, s>>>(faces, n, tslots, n_parts, lamda, lam_y, max_iter, stop, votes,
                                                     vote_counts, ms_mean, out, 1);
  if (which == 1) {
    if (FFD_MS_SORT && order) {  // chains sorted by list length, MS_FACES per workgroup
      k_ms_order<<<1, 1024, 0, s>>>(faces, n, n_parts, vote_counts, order);
      const dim3 grid((unsigned)((chains + MS_FACES - 1) / MS_FACES));
      k_meanshift<<<grid, MS_THREADS, 0, s>>>(faces, n, tslots, n_parts, lamda, lam_y, max_iter, stop, votes, vote_counts, ms_mean,
                                    out, order);
    } else {
      const dim3 grid((n + MS_FACES - 1) / MS_FACES, NPARTS);
      k_meanshift<<<grid, MS_THREADS, 0, s>>>(faces, n, tslots, n_parts, lamda, lam_y, max_iter, stop, votes, vote_counts, ms_mean,
                                    out, nullptr);
    }
    return;
  }
  const int64_t lists = (int64_t)n * NPARTS;
  // wave-independent form: the most chains per wave (fewer idle lanes in the sums) that still gives
  // >= FFD_MS_WAVES waves (default 4096: four per SIMD)
  static const int64_t want = [] {
    const char* v = std::getenv("FFD_MS_WAVES");
    return v ? std::atoll(v) : (int64_t)4096;
  }();
  const int32_t* ord = nullptr;
  if (FFD_MS_SORT && order) {
    k_ms_order<<<1, 1024, 0, s>>>(faces, n, n_parts, vote_counts, order);
    ord = order;
  }
  auto launch4 = [&](int C) {
    const int64_t waves = (lists + C - 1) / C;
    const dim3 grid((unsigned)((waves + 3) / 4));
    decltype(&k_meanshift4<2, FFD_MS_K>) k;
    switch (C) {
      case 16: k = k_meanshift4<16, FFD_MS_K>; break;
      case 8: k = k_meanshift4<8, FFD_MS_K>; break;
      case 4: k = k_meanshift4<4, FFD_MS_K>; break;
      default: k = k_meanshift4<2, FFD_MS_K>; break;
    }
    k<<<grid, 256, 0, s>>>(faces, n, tslots, n_parts, lamda, lam_y, max_iter, stop, votes, vote_counts, ms_mean, out, ord);
  };
  int C = 16;
  while (C > 2 && (lists + C - 1) / C < want) C >>= 1;
  launch4(C);
}

}  // namespace ffd
