// ffd_synth_forest.cpp — synthetic FFD forest for SURVEY.md §8(d) config C4 ("deep/wide stress").
//
// Writes an FFDMODEL file whose head-pose forest is copied from a converted pretrained model and
// whose FFD side is ONE pose forest of `trees` complete trees of depth `depth` (2^depth - 1 split
// nodes and 2^depth leaves each), used for every pose bin.  Splits are drawn like
// SimplePatchFeature::generate (/root/reference/include/ImageSample.hpp:42-72): channel U{0..37},
// w, h U{1..22}, x U{0..30-w}, y U{0..30-h} for each rectangle; threshold round(N(0, 20.5^2))
// (the spread of the shipped trees' thresholds).  Leaves are random:
// samples U{3..50}, foreground U[0.3, 1), offsets U{-60..60}^2, variance U[0, 40), pf U[0, 1).
// Nodes are stored in the archive's pre-order (node, left subtree, right subtree), exactly what
// ffd_convert produces from Boost archives, so the engine and the oracle load it unchanged.
//
// usage: ffd_synth_forest <pretrained.bin> <out.bin> [depth=20] [trees=20] [seed=4]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "model_io.hpp"

using namespace ffd;

namespace {

template <typename T>
ModelArray make_array(const char* dtype, std::vector<uint64_t> shape) {
  ModelArray a;
  a.dtype = dtype;
  a.shape = std::move(shape);
  a.bytes.assign(a.count() * sizeof(T), 0);
  return a;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s <pretrained.bin> <out.bin> [depth=20] [trees=20] [seed=4]\n", argv[0]);
    return 2;
  }
  const int depth = argc > 3 ? std::atoi(argv[3]) : 20;
  const int trees = argc > 4 ? std::atoi(argv[4]) : 20;
  const uint64_t seed = argc > 5 ? std::strtoull(argv[5], nullptr, 10) : 4;
  if (depth < 1 || depth > 24 || trees < 1 || trees > 32) {
    std::fprintf(stderr, "depth must be 1..24 and trees 1..32\n");
    return 2;
  }
  try {
    ModelFile base;
    base.load(argv[1]);
    ModelFile out;
    for (const auto& kv : base.arrays)
      if (kv.first.rfind("hp.", 0) == 0) out.arrays[kv.first] = kv.second;

    const uint64_t leaves_per_tree = 1ull << depth, nodes_per_tree = 2 * leaves_per_tree - 1;
    const uint64_t N = nodes_per_tree * trees, L = leaves_per_tree * trees;
    std::vector<int32_t> param(base.get("mp.param").as<int32_t>(), base.get("mp.param").as<int32_t>() + 8);
    param[0] = depth;  // max_depth
    param[3] = trees;  // ntrees
    param[7] = 1;      // one pose forest, used for every pose bin
    out.put("mp.param", "i32", {8}, param);
    out.arrays["mp.patch_ratio"] = base.get("mp.patch_ratio");
    out.arrays["mp.features"] = base.get("mp.features");

    auto node_off = make_array<int64_t>("i64", {(uint64_t)trees + 1});
    auto leaf_off = make_array<int64_t>("i64", {(uint64_t)trees + 1});
    auto node_leaf = make_array<int32_t>("i32", {N});
    auto node_split = make_array<int16_t>("i16", {N, FFD_SPLIT_FIELDS});
    auto leaf_n = make_array<int32_t>("i32", {L});
    auto leaf_fg = make_array<float>("f32", {L});
    auto leaf_offset = make_array<int16_t>("i16", {L, 10, 2});
    auto leaf_var = make_array<float>("f32", {L, 10});
    auto leaf_pf = make_array<float>("f32", {L, 10});

    std::mt19937_64 rng(seed);
    std::uniform_int_distribution<int> ch_d(0, 37), wh_d(1, 22), n_d(3, 50), off_d(-60, 60);
    std::normal_distribution<double> thr_d(0.0, 20.5);
    std::uniform_real_distribution<float> fg_d(0.3f, 1.0f), var_d(0.0f, 40.0f), pf_d(0.0f, 1.0f);

    int32_t* nl = node_leaf.as<int32_t>();
    int16_t* sp = node_split.as<int16_t>();
    uint64_t node = 0, leaf = 0;
    for (int t = 0; t < trees; t++) {
      node_off.as<int64_t>()[t] = (int64_t)node;
      leaf_off.as<int64_t>()[t] = (int64_t)leaf;
      // pre-order walk of a complete tree: a node at depth d < depth is a split, at depth == depth a leaf
      std::vector<int> stack{0};
      while (!stack.empty()) {
        const int d = stack.back();
        stack.pop_back();
        if (d == depth) {
          nl[node] = (int32_t)leaf;
          leaf_n.as<int32_t>()[leaf] = n_d(rng);
          leaf_fg.as<float>()[leaf] = fg_d(rng);
          for (int i = 0; i < 10; i++) {
            leaf_offset.as<int16_t>()[(leaf * 10 + i) * 2] = (int16_t)off_d(rng);
            leaf_offset.as<int16_t>()[(leaf * 10 + i) * 2 + 1] = (int16_t)off_d(rng);
            leaf_var.as<float>()[leaf * 10 + i] = var_d(rng);
            leaf_pf.as<float>()[leaf * 10 + i] = pf_d(rng);
          }
          leaf++;
        } else {
          nl[node] = -1;
          int16_t* s = sp + node * FFD_SPLIT_FIELDS;
          s[0] = (int16_t)ch_d(rng);
          for (int r = 0; r < 2; r++) {
            const int w = wh_d(rng), h = wh_d(rng);
            s[1 + 4 * r] = (int16_t)std::uniform_int_distribution<int>(0, 30 - w)(rng);
            s[2 + 4 * r] = (int16_t)std::uniform_int_distribution<int>(0, 30 - h)(rng);
            s[3 + 4 * r] = (int16_t)w;
            s[4 + 4 * r] = (int16_t)h;
          }
          const long thr = std::lround(thr_d(rng));
          s[9] = (int16_t)std::max(-255L, std::min(255L, thr));
          stack.push_back(d + 1);  // right subtree (popped after the left one)
          stack.push_back(d + 1);  // left subtree
        }
        node++;
      }
    }
    node_off.as<int64_t>()[trees] = (int64_t)node;
    leaf_off.as<int64_t>()[trees] = (int64_t)leaf;
    out.arrays["mp.tree_node_off"] = std::move(node_off);
    out.arrays["mp.tree_leaf_off"] = std::move(leaf_off);
    out.arrays["mp.node_leaf"] = std::move(node_leaf);
    out.arrays["mp.node_split"] = std::move(node_split);
    out.arrays["mp.leaf_n"] = std::move(leaf_n);
    out.arrays["mp.leaf_fg"] = std::move(leaf_fg);
    out.arrays["mp.leaf_offset"] = std::move(leaf_offset);
    out.arrays["mp.leaf_var"] = std::move(leaf_var);
    out.arrays["mp.leaf_pf"] = std::move(leaf_pf);
    out.save(argv[2]);
    std::printf("wrote %s: %d trees x depth %d (%llu nodes, %llu leaves)\n", argv[2], trees, depth,
                (unsigned long long)N, (unsigned long long)L);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "ffd_synth_forest: %s\n", e.what());
    return 1;
  }
  return 0;
}
