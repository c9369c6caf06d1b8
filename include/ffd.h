/*
 * ffd.h — C-ABI of the MI355X conditional-regression-forest facial-landmark
 * engine (drop-in for the reference's FaceForest::analyzeFace hot path).
 *
 * Every entry point replaces a reference interface (paths relative to
 * /root/reference):
 *
 *   ffd_engine_create      FaceForest::FaceForest(FaceForestOptions)      src/FaceForest.cpp:15-58
 *                          (+ Forest<S>::load, include/Forest.hpp:103-153)
 *   ffd_analyze_faces      FaceForest::analyzeFace(img, bbox, Face&) per  src/FaceForest.cpp:183-258
 *                          box, batched (the reference loops faces at     src/FaceForest.cpp:175-180)
 *   ffd_analyze_faces_device  same, inputs/outputs resident in HBM (no PCIe in the timed path)
 *   ffd_extract_channels   ImageSample(img, features, true)               src/ImageSample.cpp:11-20,77-90
 *                          -> FeatureChannelFactory::extractChannel       include/FeatureChannelFactory.hpp:35-183
 *   ffd_forest_eval_leaves Forest<S>::evaluateMT over a batch of patches  include/Forest.hpp:80-90
 *                          (Tree<S>::evaluateMT, include/Tree.hpp:173-191)
 *   ffd_sample_*           ImageSample kept in HBM + Forest<S>::evaluateMT  src/ImageSample.cpp:11-20,
 *                          per patch / per grid; MeanShift::shift           include/MeanShift.hpp:41-76
 *   ffd_get_trace          per-stage intermediates of the last batch (test hook; the reference has
 *                          plotVotes/show for the same purpose, src/face_utils.cpp:348-376)
 *   ffd_engine_destroy     FaceForest::~FaceForest                        include/FaceForest.hpp:93-95
 *   ffd_last_error         the reference prints ERROR(...) and leaves is_inizialized=false
 *                          (src/FaceForest.cpp:23-56); here a status code + message
 *
 * Conventions (same as the reference):
 *   - images are BGR 8UC3 (cvtColor BGR2GRAY at src/FaceForest.cpp:196), row stride in bytes;
 *   - boxes are in image pixels and must lie inside the image (cv::Mat ROI rule);
 *   - landmarks are bbox-relative integer pixels in the order l-eye-l, l-eye-r, mouth-l,
 *     mouth-r, mouth-b, mouth-t, r-eye-l, r-eye-r, nose-l, nose-r (output/generate_report.m:13-15);
 *   - headpose is the predicted label in [-2, 2] (src/face_utils.cpp:237).
 * No exceptions cross the ABI; no allocation is visible to the caller.  One
 * engine owns one HIP stream on one device; concurrent calls need separate
 * engines (the reference's analyzeFace is not reentrant either).
 */
#ifndef FFD_H
#define FFD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  FFD_OK = 0,
  FFD_ERR_INVALID_ARGUMENT = 1,
  FFD_ERR_MODEL = 2,
  FFD_ERR_DEVICE = 3,
  FFD_ERR_OUT_OF_MEMORY = 4,
  FFD_ERR_NOT_INITIALIZED = 5,
  FFD_ERR_INTERNAL = 6,
  FFD_ERR_UNSUPPORTED = 7    /* an image sample wider than 125 columns; a detection frame over 2^18 raw candidates */
} ffd_status;

/* Human-readable meaning of a status code (call or per-face). */
const char* ffd_status_string(int32_t status);

typedef struct ffd_engine ffd_engine;

typedef struct { int32_t x, y, width, height; } ffd_rect;              /* cv::Rect */

typedef struct {                                                       /* cv::Mat 8UC3 */
  const uint8_t* bgr;
  int32_t width, height, stride;
} ffd_image;

#define FFD_NUM_LANDMARKS 10
#define FFD_MAX_TREES 32

typedef struct {                                                       /* struct Face */
  float headpose;            /* Face::headpose                       FaceForest.hpp:72 */
  float pose_variance;       /* variance from getHeadPoseVotesMT    face_utils.cpp:235-238 */
  ffd_rect bbox;             /* Face::bbox = input box              FaceForest.cpp:192 */
  int32_t points[FFD_NUM_LANDMARKS][2]; /* Face::ffd_cordinates (bbox-relative) */
  int32_t n_trees;           /* FFD trees selected for this face (20 except edge cases) */
  int32_t status;            /* FFD_OK; FFD_ERR_INVALID_ARGUMENT: box outside the image or empty scaled
                                face (the reference's CV_Assert); FFD_ERR_OUT_OF_MEMORY: scaled face over
                                2^21 rows (> 50 GB of channel planes; box h/w > 16,777).
                                A face with no head-pose patch is FFD_OK with the reference's result:
                                NaN headpose / variance, landmarks (0, 0) */
} ffd_face;

typedef struct {             /* HeadPoseEstimatorOption, include/FaceForest.hpp:34-43 */
  int32_t num_head_pose_labels;      /* 5   */
  int32_t step_size;                 /* 4   */
  float min_foreground_probability;  /* 0.5 */
} ffd_headpose_option;

typedef struct {             /* MultiPartEstimatorOption, include/FaceForest.hpp:45-58 */
  int32_t num_parts;                 /* 10   */
  int32_t step_size;                 /* 3    */
  int32_t min_samples;               /* 2    */
  float min_forground;               /* 0.5  */
  float min_pf;                      /* 0.25 */
  float max_variance;                /* 25   */
  int32_t step_size_y;               /* 0: = step_size (the reference's single step); > 0: a
                                        separate y step (SURVEY.md C4's 4x density grid, (2, 1)) */
} ffd_multipart_option;

typedef struct {             /* MeanShiftOption, include/MeanShift.hpp:16-25 */
  int32_t kernel_size;               /* 10   */
  int32_t max_iterations;            /* 7    */
  float stopping_criteria;           /* 0.05 */
} ffd_meanshift_option;

typedef struct {
  const char* model_path;    /* FFDMODEL file written by ffd_convert (replaces tree_path dirs) */
  int32_t device;            /* HIP device ordinal */
  int32_t max_chunk_faces;   /* faces per pipeline chunk; 0 = default */
  ffd_headpose_option hp_option;
  ffd_multipart_option mp_option;
  ffd_meanshift_option ms_option;
} ffd_engine_desc;

/* Fill desc with the reference defaults (identical values to the option structs' ctors). */
void ffd_engine_desc_init(ffd_engine_desc* desc);

ffd_status ffd_engine_create(const ffd_engine_desc* desc, ffd_engine** out);
void ffd_engine_destroy(ffd_engine* engine);
/* Last error message for this engine (or for a failed create when engine == NULL). */
const char* ffd_last_error(const ffd_engine* engine);

/* Scaled-face geometry of a box (FaceForest.cpp:202-204; face_utils.cpp:197-207,255-265). */
ffd_status ffd_face_geometry(const ffd_engine* engine, int32_t box_w, int32_t box_h, int32_t* face_w,
                             int32_t* face_h, int32_t* n_hp_patches, int32_t* n_mp_patches);

/* analyzeFace for n_faces boxes; face i uses imgs[box_img[i]] (box_img may be NULL when
 * n_img == n_faces: face i on image i).  Host buffers in, host results out. */
ffd_status ffd_analyze_faces(ffd_engine* engine, const ffd_image* imgs, int32_t n_img,
                             const ffd_rect* boxes, const int32_t* box_img, int32_t n_faces,
                             ffd_face* out);

/* Same with device-resident data: d_images holds n_img images of identical geometry
 * (width, height, stride; image k at byte offset k*image_bytes); boxes/box_img are host
 * metadata; results are written to the device array d_out (n_faces ffd_face).  The call
 * is enqueued on the engine's stream and returns when the work has been queued, except
 * for one small device->host read of the per-batch tree count.  ffd_synchronize waits. */
ffd_status ffd_analyze_faces_device(ffd_engine* engine, const void* d_images, int64_t image_bytes,
                                    int32_t width, int32_t height, int32_t stride, int32_t n_img,
                                    const ffd_rect* boxes, const int32_t* box_img, int32_t n_faces,
                                    void* d_out);
ffd_status ffd_synchronize(ffd_engine* engine);
/* Opaque hipStream_t of the engine (for callers that order their own work after it). */
void* ffd_stream(ffd_engine* engine);

/* ImageSample channels for one scaled gray face (face_w x face_h, row-major, no padding):
 * out receives 38 integral planes of (face_h+1) x (face_w+1) u32 (same values as the
 * reference's CV_32F integrals, which are exact integers). */
ffd_status ffd_extract_channels(ffd_engine* engine, const uint8_t* gray_face, int32_t face_w,
                                int32_t face_h, uint32_t* out);

#define FFD_FOREST_HEADPOSE 0
#define FFD_FOREST_FFD 1

/* Forest<S>::evaluateMT over n_patches patches (top-left x,y pairs; 31x31 patches) of one
 * image sample given as 38 integral planes (layout of ffd_extract_channels).  tree_ids:
 * head-pose tree index (0..14) or FFD global tree id (forest*20 + tree).  leaf_ids[p*n_trees+t]
 * receives the global leaf ordinal reached (model file order). */
ffd_status ffd_forest_eval_leaves(ffd_engine* engine, int32_t forest_kind, const uint32_t* channels,
                                  int32_t face_w, int32_t face_h, const int32_t* patches_xy,
                                  int32_t n_patches, const int32_t* tree_ids, int32_t n_trees,
                                  int32_t* leaf_ids);

/* FaceForest::estimateHeadPose (static, include/FaceForest.hpp:97-105, src/FaceForest.cpp:60-72 ->
 * getHeadPoseVotesMT, src/face_utils.cpp:183-242) on an image sample given as 38 integral planes
 * (layout of ffd_extract_channels), patches over `region` (the reference's face_bbox; NULL = the
 * whole sample), with the call's HeadPoseEstimatorOption (NULL = the engine's desc->hp_option):
 * step_size, num_head_pose_labels and min_foreground_probability all apply.  headpose / variance as
 * Face::headpose and getHeadPoseVotesMT's variance. */
ffd_status ffd_estimate_headpose(ffd_engine* engine, const uint32_t* channels, int32_t face_w, int32_t face_h,
                                 const ffd_rect* region, const ffd_headpose_option* options, float* headpose,
                                 float* variance);

/* FaceForest::estimateFacialFeatures (static, include/FaceForest.hpp:107-115, src/FaceForest.cpp:74-95):
 * the FFD forest made of the given global tree ids (forest*20 + tree, at most FFD_MAX_TREES), votes over
 * the patches of `region` (getFacialFeaturesVotesMT, src/face_utils.cpp:244-302) under the call's
 * MultiPartEstimatorOption (NULL = the engine's desc->mp_option; every field applies), then
 * MeanShift::shift with a default MeanShiftOption as the reference does; points[2*i], points[2*i+1] =
 * landmark i in sample coordinates (cvRound), (0, 0) for i >= num_parts. */
ffd_status ffd_estimate_facial_features(ffd_engine* engine, const uint32_t* channels, int32_t face_w,
                                        int32_t face_h, const ffd_rect* region, const int32_t* tree_ids,
                                        int32_t n_trees, const ffd_multipart_option* options, int32_t* points);

/* Leaf payloads by model leaf ordinal (the ids ffd_forest_eval_leaves returns): what the reference's
 * callers read through the Leaf* of Forest<S>::evaluateMT (src/face_utils.cpp:223-228, 289-295).
 * Host-side copies from the model file (read on first use); out is an array of n ffd_headpose_leaf
 * (forest_kind FFD_FOREST_HEADPOSE) or ffd_mp_leaf (FFD_FOREST_FFD). */
#define FFD_NUM_HP_LABELS_MAX 5
typedef struct {             /* HeadPoseLeaf, include/HeadPoseSample.hpp:144-162 */
  int32_t hp_nsamples;
  float hp_foreground;
  int32_t hp_labels[FFD_NUM_HP_LABELS_MAX];
} ffd_headpose_leaf;
typedef struct {             /* MPLeaf, include/MPSample.hpp:137-159 */
  int32_t mp_samples;
  float mp_foreground;
  int32_t mp_parts_offset[FFD_NUM_LANDMARKS][2];
  float mp_parts_variance[FFD_NUM_LANDMARKS];
  float mp_prob_foreground[FFD_NUM_LANDMARKS];
} ffd_mp_leaf;
ffd_status ffd_forest_leaves(ffd_engine* engine, int32_t forest_kind, const int32_t* leaf_ids, int32_t n, void* out);
/* The leaf ordinals of one tree (global tree id as in tree_ids): [*first, *first + *count).  What the reference holds
 * in memory per loaded tree (Forest::load, include/Forest.hpp:103-129); the C++ header fills a forest's payloads tree
 * by tree with it. */
ffd_status ffd_forest_tree_leaves(ffd_engine* engine, int32_t forest_kind, int32_t tree_id, int32_t* first,
                                  int32_t* count);

/* ---- Device-resident image samples (ImageSample + Forest<S>::evaluateMT, the reference's low-level API) ----
 * ffd_sample_create      ImageSample(img, features, use_integral)     src/ImageSample.cpp:11-20,77-90: the 38
 *                        integral channels of an 8-bit gray face computed on the GPU and KEPT in HBM (u16 planes
 *                        mod 2^16, exact for every rectangle a split reads); no host copy is made.
 * ffd_sample_eval_leaves Forest<S>::evaluateMT(const S*, S::Leaf**)   include/Forest.hpp:80-90 for patches of the
 *                        sample: one launch writing the leaf ordinals to pinned host memory and one stream
 *                        synchronisation (no upload, no allocation, no host narrowing per call).
 * ffd_sample_eval_grid   the same for the patch grid x0 + i*step, y0 + j*step (i < nx, j < ny): the patches
 *                        getHeadPoseVotesMT / getFacialFeaturesVotesMT (src/face_utils.cpp:197-207,255-265)
 *                        evaluate one by one, in ONE launch; leaf_ids[(i*ny + j)*n_trees + t].
 * ffd_sample_estimate_headpose / ffd_sample_estimate_facial_features: FaceForest::estimateHeadPose /
 *                        estimateFacialFeatures (static, src/FaceForest.cpp:60-95) on the sample, as
 *                        ffd_estimate_headpose / ffd_estimate_facial_features.
 * ffd_meanshift          MeanShift::shift (include/MeanShift.hpp:41-76) of one vote list on the GPU: votes
 *                        with check == 0 are skipped as in getMean / getWeightedMean; result = the mode before
 *                        rounding (the reference's Point_<int> result is cvRound of it).
 * A sample belongs to the engine that made it.  Destroying the engine first frees the sample's planes; the
 * sample's calls then fail with FFD_ERR_INVALID_ARGUMENT and ffd_sample_destroy still releases it.  Samples
 * whose integrals may pass 2^24 (255 W H >= 2^24: the reference's CV_32F integrals round) keep the rounded
 * values and are walked with the reference's float rectangle means.  Samples wider than 125 columns are
 * FFD_ERR_UNSUPPORTED (the u16 planes' pitch). */
typedef struct ffd_sample ffd_sample;
ffd_status ffd_sample_create(ffd_engine* engine, const uint8_t* gray, int32_t width, int32_t height, int32_t stride,
                             ffd_sample** out);
/* from 38 integral planes in the layout of ffd_extract_channels (e.g. the reference's own channels) */
ffd_status ffd_sample_create_from_channels(ffd_engine* engine, const uint32_t* channels, int32_t width,
                                           int32_t height, ffd_sample** out);
void ffd_sample_destroy(ffd_sample* sample);
ffd_status ffd_sample_size(const ffd_sample* sample, int32_t* width, int32_t* height);
/* the channels back as 38 u32 integral planes (ffd_extract_channels layout) */
ffd_status ffd_sample_channels(const ffd_sample* sample, uint32_t* out);
ffd_status ffd_sample_eval_leaves(ffd_sample* sample, int32_t forest_kind, const int32_t* patches_xy,
                                  int32_t n_patches, const int32_t* tree_ids, int32_t n_trees, int32_t* leaf_ids);
ffd_status ffd_sample_eval_grid(ffd_sample* sample, int32_t forest_kind, int32_t x0, int32_t y0, int32_t step,
                                int32_t nx, int32_t ny, const int32_t* tree_ids, int32_t n_trees, int32_t* leaf_ids);
ffd_status ffd_sample_estimate_headpose(ffd_sample* sample, const ffd_rect* region, const ffd_headpose_option* options,
                                        float* headpose, float* variance);
ffd_status ffd_sample_estimate_facial_features(ffd_sample* sample, const ffd_rect* region, const int32_t* tree_ids,
                                               int32_t n_trees, const ffd_multipart_option* options, int32_t* points);
typedef struct {             /* Vote, include/face_utils.hpp:34-42 */
  int32_t x, y;              /* pos */
  float weight;
  int32_t check;
} ffd_vote;
ffd_status ffd_meanshift(ffd_engine* engine, const ffd_vote* votes, int32_t n, const ffd_meanshift_option* option,
                         float* mean_xy);

/* Intermediates of face `index` of the most recent ffd_analyze_faces[_device] batch.
 * Any pointer may be NULL; sizes as documented per field (from ffd_face_geometry). */
typedef struct {
  uint8_t* face;         /* face_w*face_h scaled gray face                          */
  uint32_t* channels;    /* 38*(face_h+1)*(face_w+1) integral channels              */
  int32_t* hp_leaves;    /* n_hp_patches*15, [patch][tree], reference patch order   */
  int32_t* mp_leaves;    /* n_mp_patches*n_trees, [patch][tree]                     */
  int32_t* trees;        /* FFD_MAX_TREES selected global FFD tree ids (n_trees used) */
  float* pose_freq;      /* 5 areaUnderCurve values                                 */
  int32_t* vote_counts;  /* 10 votes per landmark                                   */
  float* ms_mean;        /* 20: MeanShift mode (x,y) per landmark before rounding   */
} ffd_trace;

ffd_status ffd_get_trace(ffd_engine* engine, int32_t index, ffd_trace* trace);

/* Diagnostic: the Gabor kernels' branch-free magnitude sqrt (mag_sqrt, csrc/ffd_kernels.hip) checked
 * on the device against sqrtf for every float of its exact domain (+0 and all finite s >= 2^-96);
 * magnitudes outside it make the fast Gabor pass hand the face to its exact (sqrtf) instance. */
ffd_status ffd_check_mag_sqrt(ffd_engine* engine, uint64_t* checked, uint64_t* mismatches);

/* Per-stage device time of the pipeline, measured with hipEvents on the engine stream
 * (kernel boundaries only; used by bench.py for the roofline of the dominant kernel).
 * ffd_set_profiling(e, 1) enables and resets the accumulators. */
#define FFD_NUM_STAGES 12
ffd_status ffd_set_profiling(ffd_engine* engine, int32_t enable);
ffd_status ffd_get_stage_times(ffd_engine* engine, double* total_ms, int64_t* launches, int32_t n_stages);
const char* ffd_stage_name(int32_t stage);

/* ---- multi-device ----------------------------------------------------------
 * Faces are independent (the reference loops them, src/FaceForest.cpp:175-180): each device keeps
 * its own copy of the model, owns a contiguous block of ceil(N / G) faces and runs the whole path on
 * it; the ffd_face records are gathered to one device with ONE RCCL gather over xGMI. */

/* One process, G devices: an engine per device (desc->device is ignored) + ncclCommInitAll. */
typedef struct ffd_group ffd_group;
ffd_status ffd_group_create(const ffd_engine_desc* desc, const int32_t* devices, int32_t n_devices, ffd_group** out);
void ffd_group_destroy(ffd_group* group);
const char* ffd_group_last_error(const ffd_group* group);  /* group == NULL: the last failed create */
int32_t ffd_group_size(const ffd_group* group);
ffd_engine* ffd_group_engine(ffd_group* group, int32_t index);  /* owned by the group */
/* analyzeFace over n_faces boxes sharded over the devices; same arguments and results as
 * ffd_analyze_faces (out: host array, face order preserved). */
ffd_status ffd_group_analyze_faces(ffd_group* group, const ffd_image* imgs, int32_t n_img, const ffd_rect* boxes,
                                   const int32_t* box_img, int32_t n_faces, ffd_face* out);

/* Test hook: the group's per-device driver (one host thread per device) running n tasks that each sleep
 * `ms` milliseconds; *wall_ms is the elapsed time (about ms when the devices' work is issued concurrently). */
ffd_status ffd_group_debug_overlap(int32_t n, int32_t ms, double* wall_ms);

/* One process per device: one rank creates the id (ncclGetUniqueId) and shares it with the others
 * (MPI / torch.distributed broadcast, a file ...); every rank joins with its engine
 * (ncclCommInitRank on the engine's device); ffd_gather_faces then gathers n_per_rank ffd_face
 * records from every rank's device buffer d_local into d_root (n_ranks * n_per_rank records, rank
 * order) on rank `root`, enqueued on the engine's stream (after its pending batch). */
#define FFD_COMM_ID_BYTES 128
ffd_status ffd_comm_id(uint8_t* id /* FFD_COMM_ID_BYTES */);
ffd_status ffd_engine_join(ffd_engine* engine, const uint8_t* id, int32_t n_ranks, int32_t rank);
ffd_status ffd_gather_faces(ffd_engine* engine, const void* d_local, int32_t n_per_rank, void* d_root, int32_t root);
/* The joined communicator's size and this engine's rank as RCCL reports them (ncclCommCount /
 * ncclCommUserRank); FFD_ERR_NOT_INITIALIZED when the engine has not joined. */
ffd_status ffd_engine_comm_info(ffd_engine* engine, int32_t* n_ranks, int32_t* rank);

/* ---- Haar face detector and the frame-level API ---------------------------
 * ffd_detect_faces      FaceForest::detectFace   src/FaceForest.cpp:136-159: the model's Haar cascade
 *                       (ffd_convert reads data/haarcascade_frontalface_alt.xml) run as OpenCV 2.4.9's
 *                       CascadeClassifier::detectMultiScale(frame, boxes, search_scale_factor,
 *                       min_neighbors, 0, Size(min_feature_size, min_feature_size)), then the 5 % / 15 %
 *                       widening clipped to the frame; on the GPU, every frame of the batch at once.
 * ffd_analyze_images    FaceForest::analyzeImage src/FaceForest.cpp:161-181: detect, then analyzeFace on
 *                       every box (all boxes of all frames as one batch); faces in frame order, then
 *                       detection order; face_img[i] = the frame of face i.
 * Boxes beyond max_boxes / max_faces are counted in *n_boxes / *n_faces but not written.
 * Frames are grouped on the GPU with up to 8,192 raw (ungrouped) detections each in LDS; a frame with more
 * (natural 1080p frames give a few hundred) is run again on its own with a capacity that holds all of them
 * (component labels in global memory, the pair tests spread over every CU; measured whole-frame detection: a
 * 3840 x 2160 frame with 39,521 raw detections 0.13 s, a 7680 x 4320 one with 167,103 0.67 s); a frame with more
 * than 2^18 raw detections (about 1.6 s of grouping) fails with FFD_ERR_UNSUPPORTED.
 * Parity: bit-exact with the CPU restatement (oracle/); with OpenCV itself unpinned (no OpenCV here). */
typedef struct {
  int32_t min_feature_size;    /* FaceDetectionOption (include/FaceForest.hpp:21-32): 30 */
  int32_t min_neighbors;       /* 1 (0: the raw, ungrouped detections) */
  float search_scale_factor;   /* 1.3f */
  int32_t widen;               /* 1: detectFace's enlargement + clip; 0: detectMultiScale's boxes */
} ffd_detect_options;
void ffd_detect_options_init(ffd_detect_options* opt);
ffd_status ffd_detect_faces(ffd_engine* engine, const ffd_image* imgs, int32_t n_img, const ffd_detect_options* opt,
                            ffd_rect* boxes, int32_t* box_img, int32_t max_boxes, int32_t* n_boxes);
/* frames already in HBM: n_img frames of one size, image_bytes apart */
ffd_status ffd_detect_faces_device(ffd_engine* engine, const void* d_images, int64_t image_bytes, int32_t width,
                                   int32_t height, int32_t stride, int32_t n_img, const ffd_detect_options* opt,
                                   ffd_rect* boxes, int32_t* box_img, int32_t max_boxes, int32_t* n_boxes);
ffd_status ffd_analyze_images(ffd_engine* engine, const ffd_image* imgs, int32_t n_img, const ffd_detect_options* opt,
                              ffd_face* faces, int32_t* face_img, int32_t max_faces, int32_t* n_faces);
/* FaceForest::detectFace with the CascadeClassifier it is given (include/FaceForest.hpp:125-132, the static
 * overload): an engine that holds only the Haar cascade of an OpenCV XML file (BOOST / HAAR stumps, the
 * converter's reader) on `device`, for ffd_detect_faces / ffd_detect_faces_device / ffd_detect_candidates.
 * The forest entry points fail on it (FFD_ERR_INVALID_ARGUMENT).  A missing or malformed file fails
 * (FFD_ERR_MODEL), as CascadeClassifier::load returns false.  Destroy with ffd_engine_destroy. */
ffd_status ffd_detector_create(const char* cascade_xml, int32_t device, ffd_engine** out);
/* test hook: detectMultiScale's ungrouped candidates of one frame, in scan order */
ffd_status ffd_detect_candidates(ffd_engine* engine, const ffd_image* img, const ffd_detect_options* opt,
                                 ffd_rect* raw, int32_t cap, int32_t* n_raw);

/* ---- Boost text-archive writer ------------------------------------------
 * Replaces Tree<S>::save (include/Tree.hpp:239-256: boost::archive::text_oarchive << *this) and the
 * serializers it runs (Tree.hpp:336-343, Constants.hpp:44-59, TreeNode.hpp:150-164,
 * ThresholdSplit.hpp:60-67, ImageSample.hpp:83-90, MPSample.hpp:149-158, HeadPoseSample.hpp:154-161):
 * re-emits a tree of an FFDMODEL container as the reference's archive bytes (the converted
 * pretrained trees byte-for-byte equal to the shipped files).  Host only; no device needed.
 * Tree index t of FFD_FOREST_FFD is forest-major (forest t / ntrees, tree t % ntrees). */
typedef struct ffd_model ffd_model;
ffd_status ffd_model_open(const char* path, ffd_model** out);
void ffd_model_close(ffd_model* model);
const char* ffd_model_last_error(void);  /* this thread's last ffd_model_* failure */
int32_t ffd_model_num_trees(const ffd_model* model, int32_t forest_kind);
/* the tree's archived m_save_path (Tree.hpp:254: where Tree<S>::save writes) */
ffd_status ffd_model_tree_save_path(const ffd_model* model, int32_t forest_kind, int32_t tree, char* buf, int32_t cap);
/* the archive bytes into buf (buf == NULL: only *size); not NUL-terminated */
ffd_status ffd_model_tree_archive(const ffd_model* model, int32_t forest_kind, int32_t tree, char* buf, int64_t cap,
                                  int64_t* size);
ffd_status ffd_model_save_tree(const ffd_model* model, int32_t forest_kind, int32_t tree, const char* path);

/* ---- Model conversion (the reference's FaceForest ctor / Forest<S>::load inputs) -------------------
 * ffd_model_convert  FaceForest::FaceForest's loads (src/FaceForest.cpp:15-58): hp->ntrees head-pose trees
 *                    from hp->tree_path, mp->ntrees trees from each of mp_dirs (in the given order; the
 *                    reference sorts the sub-directories of mp_forest_param.tree_path, FaceForest.cpp:39-45,
 *                    which ffd_forest_subdirs lists), through Forest<S>::load / Tree<S>::load
 *                    (include/Forest.hpp:103-153, Tree.hpp:193-237), and the Haar cascade XML (may be NULL),
 *                    into the FFDMODEL file ffd_engine_create loads.  Host only.
 * ffd_forest_subdirs the sorted sub-directories of dir, NUL-separated, into buf (NULL: only *size). */
typedef struct {                 /* ForestParam, include/Constants.hpp:24-60 */
  int32_t max_depth, min_patches, ntests, ntrees, nimages, npatches, face_size;
  float patch_size_ratio;
  const char* tree_path;
  const char* image_path;
  const int32_t* features;
  int32_t n_features;
} ffd_forest_param;
ffd_status ffd_model_convert(const ffd_forest_param* hp, const ffd_forest_param* mp, const char* const* mp_dirs,
                             int32_t n_mp_dirs, const char* cascade_xml, const char* out_path);
const char* ffd_model_convert_last_error(void);  /* this thread's last ffd_model_convert / ffd_forest_subdirs failure */
ffd_status ffd_forest_subdirs(const char* dir, char* buf, int64_t cap, int64_t* size);

/* ---- Facial-feature tree training ----------------------------------------
 * Replaces trainTree (src/train_ffd.cpp:34-123) from the training ROIs on: the patch sampling, the
 * MPSample ctor (src/MPSample.cpp:13-41), Tree<MPSample>(samples, param, rng, save_path)
 * (include/Tree.hpp:43-63) with grow / findOptimalSplit / applyOptimalSplit (Tree.hpp:102-171,261-308),
 * SplitGen::generate / generateMT / findThreshold / splitSamples (include/SplitGen.hpp:62-231) and
 * MPSample::generateSplit / evalSplit / makeLeaf (src/MPSample.cpp:86-297).  The split search of every
 * node of a tree level runs on the GPU (one wave per (node, stripe)); the result is the reference's
 * Tree archive (Tree<S>::save, Tree.hpp:239-256) through the writer above.
 * Seeds: tree_seed is trainTree's rng.seed(idx_tree + 1); split_seed stands for the std::time(NULL) of
 * SplitGen::generateMT (SplitGen.hpp:78), which makes the reference's training irreproducible: stripe s
 * of the node with heap index h (root 1, children 2h, 2h + 1) uses mt19937((s + 1) * (split_seed + h)).
 * Definitions the reference leaves open are listed in oracle/ffd_train_oracle.cpp (parity unpinned). */
typedef struct {                 /* ForestParam, include/Constants.hpp:24-60 (config_ffd.txt values) */
  int32_t max_depth;             /* 20 */
  int32_t min_patches;           /* 20 */
  int32_t ntests;                /* 2500 */
  int32_t ntrees;                /* 20  (archived) */
  int32_t nimages;               /* 600 (archived) */
  int32_t npatches;              /* 150 patches per image */
  int32_t face_size;             /* 125 */
  float patch_size_ratio;        /* 0.25: patch size round(face_size * ratio) = 31 */
  const char* tree_path;         /* archived ForestParam::tree_path ("data/trees_ffd") */
  const char* image_path;        /* archived ForestParam::image_path */
  const char* save_path;         /* archived Tree::m_save_path */
  uint32_t tree_seed;            /* rng.seed(idx_tree + 1), train_ffd.cpp:66-67 */
  uint32_t split_seed;           /* std::time(NULL)'s stand-in, see above */
  int32_t device;                /* HIP device ordinal */
} ffd_train_param;

typedef struct {                 /* one training image: the ROI of train_ffd.cpp:82-99 */
  const uint8_t* gray;           /* enlarged face at face_size scale, 8-bit gray */
  int32_t width, height, stride;
  const int32_t* parts;          /* 10 x (x, y) landmarks in ROI pixels (annotations[i].parts) */
} ffd_train_image;

typedef struct {                 /* where the time went (host wall clock, ms) */
  double channels_ms, search_ms, partition_ms, leaves_ms, total_ms;
  int64_t samples, items;        /* patches; (node, stripe) items evaluated over all levels */
  int32_t levels;
} ffd_train_stats;

typedef struct ffd_trained_tree ffd_trained_tree;

void ffd_train_param_init(ffd_train_param* p);
ffd_status ffd_train_mp_tree(const ffd_train_param* p, const ffd_train_image* images, int32_t n_images,
                             ffd_trained_tree** out);
/* the same with the caller's patches instead of npatches draws per image: n_patches (image, x, y) triples, each a
 * face_size * patch_size_ratio square inside its image (Tree<MPSample>(samples, param, rng, save_path) of a caller
 * that made its MPSamples itself, include/Tree.hpp:43-64, src/demo.cpp:48-100); tree_seed is then unused */
ffd_status ffd_train_mp_tree_patches(const ffd_train_param* p, const ffd_train_image* images, int32_t n_images,
                                     const int32_t* patches, int64_t n_patches, ffd_trained_tree** out);
const char* ffd_train_last_error(void);  /* this thread's last ffd_train_* failure */
int64_t ffd_trained_tree_num_nodes(const ffd_trained_tree* t);
int64_t ffd_trained_tree_num_leaves(const ffd_trained_tree* t);
/* pre-order node arrays in the FFDMODEL layout (node_leaf: leaf ordinal or -1; node_split: channel, rect1,
 * rect2, threshold as 10 x i16; node_info: the split's information gain) and the MPLeaf payloads
 * (leaf_offset: 10 x (x, y) i16, leaf_var / leaf_pf: 10 x f32); samples_xy: (image, x, y) per patch.
 * Any pointer may be NULL. */
ffd_status ffd_trained_tree_arrays(const ffd_trained_tree* t, int32_t* node_leaf, int16_t* node_split,
                                   double* node_info, int32_t* leaf_n, float* leaf_fg, int16_t* leaf_offset,
                                   float* leaf_var, float* leaf_pf, int32_t* samples_xy);
ffd_status ffd_trained_tree_stats(const ffd_trained_tree* t, ffd_train_stats* stats);
/* Tree<MPSample>::save's (Tree<HeadPoseSample>::save's) archive bytes (buf == NULL: only *size) / to a file */
ffd_status ffd_trained_tree_archive(const ffd_trained_tree* t, char* buf, int64_t cap, int64_t* size);
ffd_status ffd_trained_tree_save(const ffd_trained_tree* t, const char* path);
void ffd_trained_tree_free(ffd_trained_tree* t);

/* ---- Head-pose tree training -------------------------------------------------
 * Replaces train_headpose.cpp's trainTree (src/train_headpose.cpp:40-143) from the scaled images on:
 * positive / negative patch sampling (:98-134), Tree<HeadPoseSample> growth with the reference's
 * split-mode draw per searched node (include/Tree.hpp:102-171,261-289) and HeadPoseSample::generateSplit /
 * evalSplit / entropie / gain2 / makeLeaf (src/HeadPoseSample.cpp:48-248).  The mode of a node is the
 * tree generator's next draw in DEPTH-FIRST order, so nodes are searched one at a time in that order
 * (every stripe of the node in parallel on the GPU), not a level at a time.  Seeds as above.
 * ffd_trained_tree_archive / _save give Tree<HeadPoseSample>::save's archive for such a tree. */
typedef struct {                 /* one training image of train_headpose.cpp:83-96 */
  const uint8_t* gray;           /* the whole image, scaled so the face box is face_size wide, 8-bit gray */
  int32_t width, height, stride;
  ffd_rect face;                 /* annotations[i].bbox after the scaling; positives lie in
                                    [face.x, face.x + face_size - 1) x [face.y, face.y + face_size - 1) */
  int32_t pose;                  /* annotations[i].pose in [-2, 2] (label pose + 2) */
} ffd_train_hp_image;

void ffd_train_hp_param_init(ffd_train_param* p);  /* config_headpose.txt: depth 15, 2000 tests, 200 patches */
ffd_status ffd_train_hp_tree(const ffd_train_param* p, const ffd_train_hp_image* images, int32_t n_images,
                             ffd_trained_tree** out);
int32_t ffd_trained_tree_kind(const ffd_trained_tree* t);          /* FFD_FOREST_FFD or FFD_FOREST_HEADPOSE */
int64_t ffd_trained_tree_num_samples(const ffd_trained_tree* t);   /* sampled patches */
/* A head-pose tree's pre-order arrays (node_mode: the split mode drawn for each split node, -1 for a
 * leaf), HeadPoseLeaf payloads (leaf_labels: 5 x i32 per leaf) and patches (image, x, y, label; label -1
 * for background).  Any pointer may be NULL. */
ffd_status ffd_trained_tree_hp_arrays(const ffd_trained_tree* t, int32_t* node_leaf, int16_t* node_split,
                                      double* node_info, int32_t* node_mode, int32_t* leaf_n, float* leaf_fg,
                                      int32_t* leaf_labels, int32_t* samples);

/* Library version string. */
const char* ffd_version(void);

#ifdef __cplusplus
}
#endif

#endif /* FFD_H */
