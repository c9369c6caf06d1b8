// ffd_haar.hpp — data layout and launchers of the Haar face detector (ffd_haar.hip), shared by the
// kernels and the host orchestration (ffd_detect.cpp).  SURVEY.md §8(f) #1: FaceForest::detectFace,
// /root/reference/src/FaceForest.cpp:136-159.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

namespace ffd {

constexpr int HAAR_MAX_CAND = 8192;  // raw candidates per frame the grouping kernel holds (LDS labels)
// raw candidates of one frame grouped at all (FFD_ERR_UNSUPPORTED beyond): the min-label rounds' pair tests grow as
// N^2; measured whole-frame detection 0.67 s at 167,103 (tools/r5_haar_bign.py), so ~1.6 s at this ceiling
constexpr int HAAR_GROUP_MAX = 1 << 18;

// One frame of a detection batch.
struct HaarFrame {
  int64_t img_off;   // BGR bytes in the image buffer
  int64_t gray_off;  // its gray copy (pitch w)
  int32_t w, h, stride;
  int32_t level0, level1;  // its pyramid levels [level0, level1)
  int32_t rows;            // scan rows over all its levels
};

// One pyramid level (frame, scale factor) that detectMultiScale scans.
struct HaarLevel {
  int64_t gray_off;  // source gray frame (pitch src_w)
  int64_t img_off;   // scaled image (pitch sw)
  int64_t sum_off;   // integral sum / sqsum ((sh + 1) x (sw + 1))
  int64_t res_off;   // per-position results (ny x nx, int8)
  double factor, scale_x, scale_y;
  int32_t src_w, src_h, sw, sh;
  int32_t ystep, nx, ny, win_w, win_h;
  int32_t mode, xv;  // resize: 0 copy, 1 bilinear, 2 area 2x; SSE2 column bound
  int32_t row0;      // first scan row of this level within its frame
  int32_t frame;
  int32_t tile0;     // the level's first cascade tile in its launch's one-dimensional grid (k_haar_cascade)
};

// One stump weak classifier with its Haar feature (HaarEvaluator::Feature + DTreeNode + 2 leaves), its
// rectangles as corner offsets into the cascade kernel's LDS window (row pitch haar_win_cols(ystep, ww),
// so one table per ystep): rect k sums win[a] - win[b] - win[c] + win[d] with a | b << 16 = o[2k],
// c | d << 16 = o[2k + 1] (the rectangle (x, y, w, h): a = y W + x, b = a + w, c = a + h W, d = c + w).
struct HaarWeak {
  uint32_t o[6];
  float w0, w1, w2;     // rect weights (w2 == 0: two-rectangle feature, rect 2 empty)
  float thr, leaf0, leaf1;
};
static_assert(sizeof(HaarWeak) == 48, "HaarWeak is 48 bytes");

struct HaarStage {
  int32_t first, ntrees;
  float thr;  // (float)stageThreshold - 1e-5f (CascadeClassifier::Data::read THRESHOLD_EPS)
  int32_t n_two;  // its first n_two classifiers are two-rectangle features (ffd_detect.cpp load_cascade)
  int32_t n_sh;   // the first n_sh of those share two corners (HAAR_SHARED records)
};
// A two-rectangle classifier whose rectangles share two corners (an edge segment): o[0] = S1 | S2 << 16 (the shared
// corners, S1 the one rect 0 adds), o[1] = X1 | X2 << 16 (rect 0's others, X2 added), o[2] = Y1 | Y2 << 16 (rect 1's,
// Y2 added), o[3] = HAAR_SHARED; w1 carries rect 1's sign.  rect 0 = E - X1 + X2, rect 1 = E - Y1 + Y2 with
// E = S1 - S2: the same integers from six corner reads instead of eight.
constexpr uint32_t HAAR_SHARED = 0xFFFFFFFFu;

void launch_haar_gray(const HaarFrame* frames, int n_frames, int max_pixels, const uint8_t* images, uint8_t* gray,
                      hipStream_t s);
void launch_haar_pyramid(const HaarLevel* levels, int n_levels, int max_pixels, int max_rows, int max_cols,
                         const uint8_t* gray, uint8_t* scaled, int32_t* sum, uint32_t* sq, hipStream_t s);
// a workgroup per 64 x 8 scan positions: max_tiles = the largest level's ceil(nx / 64) * ceil(ny / 8);
// lds_bytes = haar_cascade_lds(largest ystep of the batch, ww, wh) (dynamic LDS: the integral window)
#ifndef FFD_HAAR_TILE_Y
#define FFD_HAAR_TILE_Y 8  // scan rows per cascade workgroup tile
#endif
constexpr int HAAR_TILE_X = 64, HAAR_TILE_Y = FFD_HAAR_TILE_Y;
int haar_cascade_lds(int max_ystep, int ww, int wh);
// weak: the ystep-1 table, then (at weak + n_weak) the ystep-2 table
void launch_haar_cascade(const HaarLevel* levels, int n_levels, int total_tiles, const int32_t* sum, const uint32_t* sq,
                         const HaarWeak* weak, int n_weak, const HaarStage* stages, int n_stages, int ww, int wh,
                         int order_free, int8_t* result, int lds_bytes, hipStream_t s);
constexpr int haar_window_cols(int ystep, int ww) { return HAAR_TILE_X * ystep + ww; }
// Element (row y, column x) of a tile's LDS integral window.  ystep 2 stores the even columns, then
// the odd ones (half = ceil(cols / 2)): the 64 positions of a tile row are 2 columns apart, so a
// corner read by a wave hits consecutive words (no 2-way bank conflict), and because a corner's
// column parity is the same for every position, the offset stays position-independent:
// window(2 ly + y, 2 lx + x) = [2 ly * cols + lx] + haar_window_offset(2, cols, y, x).
constexpr int haar_window_offset(int ystep, int cols, int y, int x) {
  return y * cols + (ystep == 2 ? (x & 1) * ((cols + 1) >> 1) + (x >> 1) : x);
}
// pack every frame's boxes (cap apart) contiguously: packed[i], owner[i]; totals[0] = box count
void launch_haar_pack(int n_frames, int cap, const int4* boxes, const int32_t* n_boxes, int4* packed, int32_t* owner,
                      hipStream_t s);
// candidates (cap per frame) in scan order, then grouped + widened boxes (cap per frame);
// cls_rect: cap int4 per frame, cls_sum: 5 cap ints per frame (scratch); label_g: cap ints per frame, used when
// cap > HAAR_MAX_CAND (the component labels do not fit the LDS).  Returns HAAR_GROUP_OK, or (the overflow re-run's
// host-driven label rounds) HAAR_GROUP_HIP_ERROR / HAAR_GROUP_NO_CONVERGENCE.
enum { HAAR_GROUP_OK = 0, HAAR_GROUP_HIP_ERROR = 1, HAAR_GROUP_NO_CONVERGENCE = 2 };
int launch_haar_group(const HaarFrame* frames, int n_frames, int max_frame_rows, int32_t* rowcnt,
                       const HaarLevel* levels, const int8_t* result, int cap, int4* cand, int32_t* n_cand, int min_neighbors, int widen, int4* cls_rect, int* cls_sum,
                       int4* boxes, int32_t* n_boxes, int* label_g, hipStream_t s);

}  // namespace ffd
