// ffd_kernels.hpp — host-side declarations of the kernel launchers (ffd_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "ffd_device.hpp"

namespace ffd {

// Gabor coefficient table (floats): scale 0 (7x7, k_gabor7) = 49 taps x 16 floats
// [re0, im0, ..., re6, im6, 0, 0]; scales 1..4 = the separable factor blocks of k_gabor_sep
// (layout in ffd_kernels.hip), each 16-B aligned.
constexpr int GABOR_WIDTHS[5] = {7, 9, 13, 19, 25};
constexpr int gabor_sep_block(int R) { return (4 + 12 * (R + 1) + 16 * (2 * R + 1) + 3) / 4 * 4; }
constexpr int GABOR_OFF0 = 0;
constexpr int GABOR_OFF1 = GABOR_OFF0 + 49 * 16;
constexpr int GABOR_OFF2 = GABOR_OFF1 + gabor_sep_block(4);
constexpr int GABOR_OFF3 = GABOR_OFF2 + gabor_sep_block(6);
constexpr int GABOR_OFF4 = GABOR_OFF3 + gabor_sep_block(9);
constexpr int GABOR_COEF_TOTAL = GABOR_OFF4 + gabor_sep_block(12);
constexpr int GABOR_OFFS[5] = {GABOR_OFF0, GABOR_OFF1, GABOR_OFF2, GABOR_OFF3, GABOR_OFF4};

// max_src: the largest valid face's source box (bw x bh pixels) of the batch, 0 = unknown (the per-pixel form)
void launch_gray_resize(const FaceDesc* faces, int n, const uint8_t* images, uint8_t* gray, hipStream_t s,
                        int max_src = 0);
// Gabor scale nu (0..4): magnitudes of the 7 orientations, face-wide min-max normalisation,
// quantisation and integration of the 7 channels (one workgroup per face)
// max_h: the tallest scaled face of the batch (sizes the padded-face LDS copy)
void launch_check_mag_sqrt(uint32_t lo, uint32_t n, uint32_t* bad, int blocks, hipStream_t s);
void launch_gabor(int nu, const FaceDesc* faces, int n, int max_h, const uint8_t* gray, const float* coef, float* mag,
                  uint16_t* chan, int* redo, int force_exact, uint32_t* split_mm, hipStream_t s);
hipError_t set_gabor_lds_limit(int bytes);
// integral channels 0 (gray), 36, 37 (Sobel)
void launch_integral(const FaceDesc* faces, int n, int max_h, const uint8_t* gray, uint16_t* chan, hipStream_t s);
constexpr int TRAV_LDS_CAP = 160 * 1024;  // one traversal workgroup per CU: all of its LDS
// patch block of a traversal workgroup: gx x gy patches of one face's grid
struct TravShape {
  int gx, gy;
};
int traverse_lds_bytes(TravShape g, int step, int step_y);
bool traverse_window_fits(TravShape g, bool hp, int step, int step_y, int lds_cap);
bool traverse_shape_supported(TravShape g, bool hp);  // an instantiated k_traverse shape
// plane: the channel plane stride shared by every face of the batch; n_wg: persistent workgroups (one per CU; rounded down to a multiple of 8 XCDs)
// pairs / far: the forest's pair records (ffd_device.hpp) and far offsets; tops / top_idx: per tree
// TOP_CAP heap-ordered pair records of its top levels and their pair indices (at most top_max
// entries per tree are staged into LDS); lds_cap: dynamic LDS of a workgroup (window + tops)
void launch_traverse(bool hp, const FaceDesc* faces, int n, int bpf, TravShape g, const uint4* pairs, const uint4* tops,
                     const uint32_t* top_idx, int top_max, const uint32_t* far, const HpState* state, int ntrees_hp,
                     int step, int step_y, int64_t plane, const uint16_t* chan, int32_t* leaf_out, int n_wg,
                     int lds_cap, hipStream_t s);
hipError_t set_traverse_lds_limit(int bytes);
// the traversals of float-integral faces (FaceDesc::fint) over the 16-B node arrays
void launch_walk_fint(bool hp, const FaceDesc* faces, int n, const uint4* nodes, const int32_t* roots, int ntrees_hp,
                      const HpState* state, int step, int step_y, const uint16_t* chan, int32_t* leaf_out, hipStream_t s);
void launch_eval_patches(const uint4* nodes, const int32_t* roots, const int32_t* tree_ids, int n_trees,
                         const int32_t* patches, int n_patches, const uint16_t* chan, int64_t plane,
                         int32_t* leaf_ids, hipStream_t s, bool fint = false);
// Forest<S>::evaluateMT on a device-resident image sample (k_sample_eval): a patch list or a patch grid
constexpr int SAMPLE_INLINE = 16;  // patches passed in the argument block
struct SampleEvalArgs {
  const uint4* nodes;      // 16-B nodes (breadth-first) of the forest kind
  const int32_t* roots;    // root node per tree id
  const uint16_t* chan;    // the sample's planes: [38][H + 1][PITCH] integrals mod 2^16
  int64_t plane;           // plane stride (elements)
  int32_t* leaf_out;       // [patch][tree] leaf ordinals (device or host-mapped memory)
  const int32_t* patches;  // (x, y) pairs when n_patches > SAMPLE_INLINE and not a grid
  int n_patches, n_trees;
  int grid_ny, x0, y0, step;  // grid mode when grid_ny > 0 (n_patches = grid_nx * grid_ny)
  int fint;                // float-rounded integrals (FaceDesc::fint): rect_mean_fint
  int32_t trees[MAX_TREES];
  int32_t inl[2 * SAMPLE_INLINE];
};
void launch_sample_eval(const SampleEvalArgs& a, hipStream_t s);
void launch_hp_pose(const FaceDesc* faces, int n, const int32_t* hp_leaf, const float* hp_m, int hp_trees,
                    int n_forests, int ntrees_per_forest, HpState* state, FaceOut* out, hipStream_t s);
// leaf_rec per FFD leaf: compact (32 B) = {vote mask, fg, 10 x u16 (x - bias_x) | (y - bias_y) << 8, pad},
// else 64 B = {vote mask, fg, off[10] = x | y << 16 (int16 each), pad}
void launch_votes(const FaceDesc* faces, int n, const int32_t* mp_leaf, const uint4* leaf_rec, bool compact,
                  int bias_x, int bias_y, const HpState* state,
                  int tslots, int step, int step_y, int half_patch, int n_parts, Vote* votes, int32_t* vote_counts,
                  hipStream_t s);
void launch_meanshift(const FaceDesc* faces, int n, const HpState* state, int tslots, int n_parts, float lamda,
                      int max_iter, float stop, const Vote* votes, const int32_t* vote_counts, float* ms_mean,
                      FaceOut* out, int32_t* order, hipStream_t s, bool any_wide = false);  // any_wide: a FaceDesc::wide face

}  // namespace ffd
