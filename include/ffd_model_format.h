/*
 * ffd_model_format.h — on-disk container for the converted pretrained forests.
 *
 * The reference stores every tree as a Boost.Serialization text archive
 * (Tree::load, /root/reference/include/Tree.hpp:193-237; grammar in SURVEY.md
 * App. A).  Parsing 282 MB of text per process start is a harness cost, so the
 * converter (face_alignment_cvpr_2012_amd/csrc/ffd_convert.cpp) rewrites the
 * archives ONCE into this flat little-endian container.  Nothing is lost: the
 * node records keep the archive's pre-order, every split field and every leaf
 * payload bit-for-bit (floats are parsed exactly as text_iarchive does).
 *
 * Layout
 *   u8  magic[8]  = "FFDMODEL"
 *   u32 version   = 1
 *   u32 n_arrays
 *   ffd_array_entry entries[n_arrays]
 *   ... array payloads, each 64-byte aligned, at entry.offset (from file start)
 *
 * Arrays (prefix "hp." = head-pose forest, "mp." = the 5 pose-conditional FFD
 * forests flattened forest-major: tree g = forest*ntrees + tree):
 *   <p>.param          i32[8]  max_depth,min_patches,ntests,ntrees,nimages,
 *                              npatches,face_size,n_forests   (ForestParam,
 *                              Constants.hpp:24-60)
 *   <p>.patch_ratio    f32[1]  ForestParam::patch_size_ratio
 *   <p>.features       i32[k]  ForestParam::features (config "0 1 2")
 *   <p>.tree_node_off  i64[T+1] first node of each tree (pre-order records)
 *   <p>.tree_leaf_off  i64[T+1] first leaf of each tree
 *   <p>.node_leaf      i32[N]  leaf ordinal (global, file order) or -1
 *   <p>.node_split     i16[N,10] channel, r1.x,r1.y,r1.w,r1.h, r2.x,r2.y,
 *                              r2.w,r2.h, threshold  (ThresholdSplit /
 *                              SimplePatchFeature, ThresholdSplit.hpp:60-67,
 *                              ImageSample.hpp:83-90); zeros for leaves
 *   hp.leaf_n          i32[L]  HeadPoseLeaf::hp_nsamples
 *   hp.leaf_fg         f32[L]  HeadPoseLeaf::hp_foreground
 *   hp.leaf_labels     i32[L,5] HeadPoseLeaf::hp_labels
 *   mp.leaf_n          i32[L]  MPLeaf::mp_samples
 *   mp.leaf_fg         f32[L]  MPLeaf::mp_foreground
 *   mp.leaf_offset     i16[L,10,2] MPLeaf::mp_parts_offset (x,y)
 *   mp.leaf_var        f32[L,10] MPLeaf::mp_parts_variance
 *   mp.leaf_pf         f32[L,10] MPLeaf::mp_prob_foreground
 *
 * Archive-only fields (not used by the engine; the Boost text-archive writer
 * ffd_model_save_tree re-emits the reference's files from them, Tree.hpp:239-256):
 *   <p>.node_info         f64[N]   ThresholdSplit::info (0 for leaves)
 *   <p>.tree_counts       i64[T,2] Tree::m_num_nodes, Tree::i_node
 *   <p>.tree_param        i32[T,7] the ForestParam each archive holds (its ints)
 *   <p>.tree_ratio        f32[T]   ... and its patch_size_ratio
 *   <p>.tree_features     i32[k]   ... and its features, per tree at
 *   <p>.tree_features_off i64[T+1]
 *   <p>.tree_strings      u8[b]    tree_path, image_path, m_save_path of tree t are
 *   <p>.tree_strings_off  i64[3T+1] bytes [off[3t+j], off[3t+j+1]), j = 0, 1, 2
 *
 * Pre-order means: a node's left subtree follows it immediately, then its
 * right subtree (TreeNode::serialize, TreeNode.hpp:150-164).
 */
#ifndef FFD_MODEL_FORMAT_H
#define FFD_MODEL_FORMAT_H

#include <stdint.h>

#define FFD_MODEL_MAGIC "FFDMODEL"
#define FFD_MODEL_VERSION 1u
#define FFD_MODEL_ALIGN 64u

#define FFD_NUM_PARTS 10
#define FFD_NUM_HP_LABELS 5
#define FFD_SPLIT_FIELDS 10

typedef struct {
  char name[48];
  char dtype[8];      /* "i8","u8","i16","i32","i64","f32","f64" */
  uint32_t ndim;
  uint32_t pad_;
  uint64_t shape[4];
  uint64_t offset;    /* from file start, FFD_MODEL_ALIGN aligned */
  uint64_t nbytes;
} ffd_array_entry;

#endif /* FFD_MODEL_FORMAT_H */
