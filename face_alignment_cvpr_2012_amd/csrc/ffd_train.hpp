// ffd_train.hpp — device records and launchers of the tree-training kernels (ffd_train.hip);
// host orchestration in ffd_train.cpp.  Internal header.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/ffd_gabor.h"

namespace ffd_train {

constexpr int NCH = 38;     // ImageSample channels for features {0, 1, 2}: gray, 35 Gabor, 2 Sobel
constexpr int MT_WIN = 48;  // mt19937 outputs kept per stripe (9 feature draws + 25 thresholds + spare)
constexpr int TR_THR = 25;  // split.num_thresholds (MPSample::generateSplit, MPSample.cpp:86-101)

// one training ROI: offsets into the channel-stage buffers (elements)
struct TrImage {
  int64_t gray_off, u8_off, mag_off, v_off, ch_off;
  int32_t w, h;
};

// one MPSample patch: image and top-left corner (its part probabilities live in a [n][10] f32 array)
struct TrSample {
  int32_t img, x, y;
};

// a node of the level being split: its slice of the level's sample list, heap index (root 1) and the
// base of its stripes' sorted lists
struct TrNode {
  int32_t beg, cnt;
  uint32_t heap;
  int32_t pad;
  int64_t sorted_off;
};

// SimplePatchFeature: channel, rect1 (x, y, w, h), rect2 (x, y, w, h)
struct TrFeature {
  int32_t ch;
  int32_t r[8];
};

struct TrBest {
  double info;
  int32_t stripe, thr, k, pad;
};

struct TrItemsArgs {
  const TrNode* nodes;
  int n_items, ntests, nthr, ps, smax;
  const int32_t* list;        // level sample list (global sample ids), node slices
  const TrImage* imgs;
  const TrSample* samples;
  const float* prob;          // [samples][10] part probabilities (MPSample::m_prob)
  const uint32_t* chan;       // integral planes of every image
  const uint32_t* raw;        // [item][MT_WIN] engine outputs (k_tr_mt)
  int32_t* sorted;            // per item: the node's samples sorted by value
  double* out_info;
  int32_t* out_thr;
  int32_t* out_k;
  int* error;
};

// head pose: one node's stripes (k_hp_items) and its split (k_hp_split)
struct HpItemsArgs {
  const int32_t* list;        // the node's samples (global sample ids)
  int n;
  uint32_t T;                 // split_seed + heap index: stripe s uses mt19937((s + 1) * T)
  int mode;                   // split_mode drawn for the node (< 50: entropie, else gain2)
  int nthr, ps, smax;
  const TrImage* imgs;
  const TrSample* samples;
  const int8_t* cls;          // per sample: label 0..4, or 5 for background
  const uint32_t* chan;
  double* out_info;           // [ntests]
  int32_t* out_thr;
  int* error;
};

struct HpSplitResult {
  double info;
  int32_t stripe, thr, na, nb, ch, rect[8], ha[6], hb[6], bad, pad;
};

struct HpSplitArgs {
  int ntests;
  const double* info;
  const int32_t* thr;
  uint32_t T;
  int ps, smax;
  const int32_t* list;
  int n;
  int32_t* out;               // [n]: left side first, then the right side
  const TrImage* imgs;
  const TrSample* samples;
  const int8_t* cls;
  const uint32_t* chan;
  HpSplitResult* res;
};

void launch_channels(const TrImage* d_imgs, int n_img, int max_px, const uint8_t* gray, const ffd_gabor_sep* sep,
                     const float* taps7, uint8_t* u8, float* mag, float* vbuf, uint32_t* chan, hipStream_t s);
void launch_mt(const TrNode* nodes, int n_items, int ntests, uint32_t split_seed, uint32_t* raw, hipStream_t s);
void launch_items(const TrItemsArgs& a, hipStream_t s);
void launch_select(int n_nodes, int ntests, const double* info, const int* thr, const int* k, TrBest* best, hipStream_t s);
void launch_hp_items(const HpItemsArgs& a, int ntests, hipStream_t s);
void launch_hp_split(const HpSplitArgs& a, hipStream_t s);
void launch_partition(int n_nodes, const TrNode* nodes, const TrFeature* feats, const TrImage* imgs, const TrSample* samples,
                      const uint32_t* chan, const int32_t* list, int32_t* next, hipStream_t s);

}  // namespace ffd_train
