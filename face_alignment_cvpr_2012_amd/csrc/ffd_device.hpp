// ffd_device.hpp — data layout shared by the host engine and the HIP kernels.
//
// HBM layout (per face, row pitch PITCH elements, see DESIGN.md §Data layout):
//   gray   u8  [H][PITCH]                  scaled gray face (FaceForest.cpp:195-204)
//   mag    f32 [35][H][PITCH]              Gabor magnitudes before min-max normalisation
//   chan   u16 [38][H+1][PITCH]            integral channels mod 2^16 (ImageSample m_feature_channels;
//                                          every rectangle the trees read is exact, ffd_kernels.hip rect_mean16)
//   hpleaf i32 [n_hp][15]                  head-pose leaf ordinal per (patch, tree), reference order
//   mpleaf i32 [n_mp][T]                   FFD leaf ordinal per (patch, tree slot), reference order
//   votes  {i16 x,y; f32 w} [10][T*n_mp]   compacted votes per landmark (MeanShift input); a face whose vote
//                                          positions may leave int16 (FaceDesc::wide) has {i32 x,y; f32 w; pad}
//                                          records over twice the space
// The reference order is x-major over the patch grid (i = xi*ny + yi, face_utils.cpp:200-207),
// tree-minor; the traversal writes its leaves there, so the order-dependent consumers (head-pose
// sums, vote lists) read them contiguously.
#pragma once

#include <stdint.h>

namespace ffd {

constexpr int PITCH = 128;        // row pitch (elements) of gray/mag/channel planes; W <= 125
constexpr int NCH = 38;           // 1 gray + 35 Gabor + 2 Sobel (config "0 1 2")
constexpr int NGABOR = 35;
constexpr int NPARTS = 10;
constexpr int NHP_LABELS = 5;
constexpr int MAX_TREES = 32;     // FFD_MAX_TREES
constexpr int MAX_FACE_H = 600;   // scaled faces up to this height stage whole into the Gabor kernels' LDS (box aspect h/w <= 4.8)
// taller ones band by band (k_gabor_sep<..., TALL>).  MAX_FACE_ROWS keeps every per-face index in 32 bits
// (leaf lists n_patches x trees < 2^31); a face that tall needs > 50 GB of channel planes: FFD_ERR_OUT_OF_MEMORY
constexpr int MAX_FACE_ROWS = 1 << 21;
// Float-integral faces and samples (FaceDesc::fint) keep their CV_32F integrals modulo 2^16 and recover each rectangle
// half in the window [-2048, 63488) (ffd_kernels.hip rect_mean_fint): exact while every integral value stays below
// FINT_LIMIT (a half's rounding error is <= 2 columns x 11 row additions x 64 = 1,408 there).  Past it the call is
// refused (FFD_ERR_UNSUPPORTED): for a 125-wide face that is a box more than 539 times taller than wide.
constexpr uint64_t FINT_LIMIT = 1ull << 31;
constexpr uint32_t LEAF_BIT = 0x80000000u;

// Flattened tree node (16 B), breadth-first per tree, children adjacent:
//   x: internal -> global index of the left child (right = left + 1); leaf -> LEAF_BIT | ordinal
//   y: ch | r1w<<6 | r1h<<11 | r2w<<16 | r2h<<21
//   z: threshold (int32)
//   w: off1 | off2<<16, off = ry*PITCH + rx (patch-relative integral-image offsets)
// Source fields: ThresholdSplit<SimplePatchFeature> (ThresholdSplit.hpp:51-67,
// ImageSample.hpp:462-464) and TreeNode::left/right (TreeNode.hpp:138-141).
//
// Pair records (k_traverse): 16 bytes = the two children (c0, c1) of one internal node, each as
// a 56-bit test, plus a 16-bit offset.  Words: x = lo(c0), y = lo(c1), z = hi(c0) | off1[7:0] << 24,
// w = hi(c1) | off1[15:8] << 24, where for a split node
//   lo = x1 | y1 << 5 | x2 << 10 | y2 << 15 | thr[5:0] << 20 | ch << 26
//   hi = w1 | h1 << 5 | w2 << 10 | h2 << 15 | thr[9:6] << 20
// (rectangles patch-relative, sides 1..22, threshold 10-bit two's complement), and for a leaf
// ch = 63 (lo >= 63 << 26) with the leaf ordinal = lo[19:0] | hi << 20.  Depth-first layout per tree: the pair of
// c0's children is the next record, c1's children are off1 records ahead (off1 = 0: the 32-bit
// offset is far[pair]).  Each tree starts with a root pair (root, unused leaf).
// Source fields: ThresholdSplit<SimplePatchFeature> (ThresholdSplit.hpp:51-67, ImageSample.hpp:83-90).

// Tree tops (k_traverse): per tree, TOP_CAP pair records of its top levels in heap order: entry 0
// = the root pair, entry 1 = the root's children pair, entry 2h + s (h >= 1) = the children pair of
// node s of entry h; entries under leaves are zero (never read).  Plus each entry's pair index.
constexpr int TOP_CAP = 64;  // levels 0..6

struct FaceDesc {
  int64_t img_off;        // byte offset of the source image
  int32_t img_w, img_h, img_stride;
  int32_t bx, by, bw, bh; // face box in the image
  int32_t W, H;           // scaled face size
  float scale;            // 125.f / bw
  int32_t mode;           // 0 copy, 1 bilinear, 2 area 2x
  double scale_x, scale_y;// resize source/dest ratios (resize(), OpenCV 2.4.9)
  int32_t xv;             // columns covered by the SSE2 vertical pass
  int32_t nhx, nhy, nmx, nmy;  // patch grid sizes (step 4 / step 3)
  int64_t gray_off;       // byte offset into the gray buffer
  int64_t mag_off;        // element offset into the mag buffer
  int64_t ch_off;         // element offset into the channel buffer
  int64_t plane;          // channel plane stride (elements) = (H+1)*PITCH
  int64_t hp_off;         // element offset into the head-pose leaf buffer
  int64_t mp_off;         // element offset into the FFD leaf buffer
  int64_t vote_off;       // element offset into the vote buffer
  int32_t valid;          // 0: box rejected, face skipped (its record gets status `reject`)
  int32_t nochan;         // 1: the channel stage skips this face (channels preloaded, or never read:
                          //    no head-pose patch fits, the reference then averages 0/0)
  int32_t reject;         // ffd_status of a rejected face
  int32_t vox, voy;       // patch-grid origin in the image sample (estimateFacialFeatures' face_bbox)
  int32_t fint;           // 1: an integral value may reach 2^24 (255 W H >= 2^24, a tall face), where the
                          //    reference's CV_32F integral rounds: float-accumulated integrals, and the
                          //    traversals' exact walker k_walk_fint instead of k_traverse
  int32_t wide;           // 1: a vote position of this face may leave int16 (a face over ~32 k rows, or far leaf
                          //    offsets): its votes are VoteW records and its MeanShift runs in k_meanshift5
};

struct FaceOut {          // == ffd_face
  float headpose;
  float pose_variance;
  int32_t bbox[4];
  int32_t points[NPARTS][2];
  int32_t n_trees;
  int32_t status;
};

struct Vote {
  int16_t x, y;
  float w;
};

struct VoteW {            // the vote of a wide face (FaceDesc::wide): two Vote slots
  int32_t x, y;
  float w;
  int32_t pad;
};

struct HpState {          // per-face head-pose result + tree selection
  float headpose, variance;
  float pose_freq[8];
  int32_t n_trees;
  int32_t trees[MAX_TREES];
};

}  // namespace ffd
