/*
 * ffd_oracle.h — C API of the CPU restatement (TEST INFRASTRUCTURE ONLY).
 *
 * The oracle is the checker for the HIP product path.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load it; the
 * product library never links or calls it.
 */
#ifndef FFD_ORACLE_H
#define FFD_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORACLE_MAX_TREES 32

typedef struct {
  float headpose;       /* FaceForest::analyzeFace face.headpose */
  float pose_variance;  /* variance from getHeadPoseVotesMT */
  int32_t face_w, face_h;  /* scaled face size */
  int32_t n_trees;      /* MP trees selected */
  int32_t points[10][2];   /* bbox-relative landmarks (Face::ffd_cordinates) */
} oracle_face;

/* Optional per-stage outputs; any pointer may be NULL. Sizes (caller allocates):
 *   face        face_w*face_h u8
 *   channels    38*(face_h+1)*(face_w+1) u32
 *   hp_leaves   n_hp_patches*15 i32 (global HP leaf ordinal, [patch][tree], reference order)
 *   mp_leaves   n_mp_patches*n_trees i32 (global MP leaf ordinal, [patch][tree])
 *   trees       ORACLE_MAX_TREES i32 (global MP tree id = forest*20+tree)
 *   pose_freq   5 f32
 *   vote_counts 10 i32
 *   ms_mean     20 f32 (MeanShift result before cvRound, x,y per part)
 */
typedef struct {
  uint8_t* face;
  uint32_t* channels;
  int32_t* hp_leaves;
  int32_t* mp_leaves;
  int32_t* trees;
  float* pose_freq;
  int32_t* vote_counts;
  float* ms_mean;
} oracle_trace;

/* Estimator options (global, not thread-safe): HeadPoseEstimatorOption / MultiPartEstimatorOption
 * (include/FaceForest.hpp:34-58) and analyzeFace's MeanShiftOption (MeanShift.hpp:16-25; the
 * reference's is always the default, the engine's ffd_meanshift_option is an extension).
 * NULL restores the reference defaults. */
typedef struct {
  int32_t hp_num_labels;  /* 5 */
  int32_t hp_step;        /* 4 */
  float hp_min_fg;        /* 0.5 */
  int32_t mp_num_parts;   /* 10 */
  int32_t mp_step_x, mp_step_y;  /* 3, 3 */
  int32_t mp_min_samples; /* 2 */
  float mp_min_fg;        /* 0.5 */
  float mp_min_pf;        /* 0.25 */
  float mp_max_var;       /* 25 */
  int32_t ms_kernel;      /* 10 */
  int32_t ms_iter;        /* 7 */
  float ms_stop;          /* 0.05 */
} oracle_options;
int oracle_set_options(const oracle_options* options);
int oracle_get_options(oracle_options* options);

int oracle_load_model(const char* path);
/* Patch-grid steps (defaults 4 / 3 / 3 = the reference's options; global, not thread-safe). */
int oracle_set_steps(int32_t hp_step, int32_t mp_step_x, int32_t mp_step_y);
const char* oracle_last_error(void);

/* analyzeFace (FaceForest.cpp:183-258). threads<=1: serial; >1: reference-shaped
 * per-stage thread pools of that many threads (ThreadPool.hpp:24-64). */
int oracle_analyze_face(const uint8_t* bgr, int32_t w, int32_t h, int32_t stride,
                        int32_t bx, int32_t by, int32_t bw, int32_t bh, int32_t threads,
                        oracle_face* out, oracle_trace* trace);

/* FaceForest::estimateHeadPose / estimateFacialFeatures (FaceForest.cpp:60-95) on an image
 * sample's 38 integral planes ([c][H+1][W+1]) with patches over the region (rx, ry, rw, rh);
 * points: 10 x (x, y) cvRound'ed MeanShift modes in sample coordinates. */
int oracle_estimate_headpose(const uint32_t* channels, int32_t W, int32_t H, int32_t rx, int32_t ry, int32_t rw,
                             int32_t rh, float* headpose, float* variance);
int oracle_estimate_facial_features(const uint32_t* channels, int32_t W, int32_t H, int32_t rx, int32_t ry,
                                    int32_t rw, int32_t rh, const int32_t* tree_ids, int32_t n_trees,
                                    int32_t* points);

/* Geometry of the scaled face for a bbox of bw x bh. */
int oracle_face_geometry(int32_t bw, int32_t bh, int32_t* face_w, int32_t* face_h,
                         int32_t* n_hp_patches, int32_t* n_mp_patches);

/* FaceForest::detectFace (src/FaceForest.cpp:136-159): the Haar cascade of the loaded model over a BGR
 * frame (cvtColor, detectMultiScale(scale_factor, min_neighbors, flags 0, Size(min_size, min_size)))
 * -> boxes[cap][4] (x, y, w, h), widened and clipped like detectFace when `widen`; raw: the ungrouped
 * candidates in scan order (optional).  Parity with OpenCV unpinned (see ffd_oracle.cpp). */
int oracle_detect_faces(const uint8_t* bgr, int32_t w, int32_t h, int32_t stride, int32_t min_size,
                        int32_t min_neighbors, float scale_factor, int32_t widen, int32_t* boxes, int32_t cap,
                        int32_t* n_boxes, int32_t* raw, int32_t raw_cap, int32_t* n_raw);

/* Facial-feature tree training (oracle/ffd_train_oracle.cpp): ForestParam
 * (Constants.hpp:24-60) plus the seeds the reference takes from idx_tree and std::time(NULL). */
typedef struct {
  int32_t max_depth, min_patches, ntests, ntrees, nimages, npatches, face_size;
  float patch_size_ratio;
  int32_t num_thresholds;  /* 25 (MPSample::generateSplit) */
  uint32_t tree_seed;      /* rng.seed(idx_tree + 1) (train_ffd.cpp:66-67) */
  uint32_t split_seed;     /* stands for std::time(NULL) in SplitGen::generateMT (+ the node's heap index) */
  float lamda;             /* MPSample ctor's lamda, 0.125 */
} oracle_train_param;
typedef struct oracle_train_tree oracle_train_tree;
/* images: n_images gray training ROIs (rows packed, stride = width); parts: n_images x n_parts x (x, y). */
int oracle_train_mp_tree(const uint8_t* const* images, const int32_t* widths, const int32_t* heights,
                         const int32_t* parts, int32_t n_images, int32_t n_parts, const oracle_train_param* p,
                         oracle_train_tree** out);
int oracle_train_tree_size(const oracle_train_tree* t, int64_t* n_nodes, int64_t* n_leaves, int64_t* i_node);
/* Pre-order node arrays in the FFDMODEL layout (node_split: 10 x i16 per node) and MPLeaf payloads;
 * samples_xy: (image, x, y) of every sampled patch.  Any pointer may be NULL. */
int oracle_train_tree_get(const oracle_train_tree* t, int32_t* node_leaf, int16_t* node_split, double* node_info,
                          int32_t* leaf_n, float* leaf_fg, int16_t* leaf_offset, float* leaf_var, float* leaf_pf,
                          int32_t* samples_xy);
void oracle_train_tree_free(oracle_train_tree* t);
/* Head-pose tree training (Tree<HeadPoseSample>, train_headpose.cpp): images are the gray images already
 * scaled so the face box is face_size wide; faces: n x (x, y, w, h) in those images; poses in [-2, 2]. */
typedef struct oracle_hp_tree oracle_hp_tree;
int oracle_train_hp_tree(const uint8_t* const* images, const int32_t* widths, const int32_t* heights,
                         const int32_t* faces, const int32_t* poses, int32_t n_images, const oracle_train_param* p,
                         oracle_hp_tree** out);
int oracle_train_hp_tree_size(const oracle_hp_tree* t, int64_t* n_nodes, int64_t* n_leaves, int64_t* i_node,
                              int64_t* n_samples);
/* node_mode: the split_mode drawn for each split node (-1 for leaves); leaf_labels: 5 per leaf;
 * samples: (image, x, y, label) per patch, label -1 for background. */
int oracle_train_hp_tree_get(const oracle_hp_tree* t, int32_t* node_leaf, int16_t* node_split, double* node_info,
                             int32_t* node_mode, int32_t* leaf_n, float* leaf_fg, int32_t* leaf_labels,
                             int32_t* samples);
void oracle_train_hp_tree_free(oracle_hp_tree* t);
const char* oracle_train_last_error(void);
double oracle_log(double x);

/* Stage hooks for known-answer tests. */
int oracle_bgr2gray(const uint8_t* bgr, int32_t w, int32_t h, int32_t stride, uint8_t* gray);
int oracle_resize(const uint8_t* src, int32_t sw, int32_t sh, int32_t sstride, int32_t dw,
                  int32_t dh, uint8_t* dst);
int oracle_channels(const uint8_t* face, int32_t w, int32_t h, uint32_t* channels);
int oracle_gabor_kernel(int32_t index, float* real, float* imag, int32_t* width);
int oracle_gabor_mag(const uint8_t* face, int32_t w, int32_t h, int32_t index, float* mag);
double oracle_area_under_curve(float x1, float x2, double mean, double std_);
/* MeanShift::shift (MeanShift.hpp:41-135) of one vote list (x, y pairs, weights): the mode before cvRound. */
void oracle_meanshift(const int32_t* xy, const float* w, int32_t n, int32_t kernel, int32_t iters, float stop,
                      float* mean_xy);
double oracle_exp(double x);
float oracle_expf(float x);

#ifdef __cplusplus
}
#endif

#endif
