// Latency of the C ABI's one-sample grid evaluation (ffd_sample_eval_grid, the first evaluateMT call of a sample in
// the reference's per-patch pattern) and of its parts: ffd_synchronize (the engine's stream queries), a grid call on a
// warm sample, a fresh sample's first grid call.  Median of N calls, microseconds, one JSON line.
// build: g++ -O2 -std=c++17 -Iinclude tools/r5_sample_latency.cpp -Lface_alignment_cvpr_2012_amd/lib -lffd
//        -Wl,-rpath,$PWD/face_alignment_cvpr_2012_amd/lib -o tools/r5_sample_latency
#include <ffd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

using Clock = std::chrono::steady_clock;
static double us(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); }
static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  ffd_engine_desc d;
  ffd_engine_desc_init(&d);
  d.model_path = argv[1];
  ffd_engine* e = nullptr;
  if (ffd_engine_create(&d, &e) != FFD_OK) return 3;
  const int W = 125, H = 125, N = 200;
  std::vector<uint8_t> gray(W * H);
  for (int i = 0; i < W * H; i++) gray[i] = (uint8_t)((i * 37 + (i / W) * 11) & 255);
  std::vector<int32_t> trees(20);
  for (int t = 0; t < 20; t++) trees[t] = 20 + t;
  const int nx = (W - 31 + 2) / 3, ny = (H - 31 + 2) / 3;
  std::vector<int32_t> leaves((size_t)nx * ny * 20);
  std::vector<double> t_sync, t_warm, t_first, t_create;
  for (int k = 0; k < N; k++) {
    auto a = Clock::now();
    ffd_synchronize(e);
    t_sync.push_back(us(a, Clock::now()));
  }
  ffd_sample* s = nullptr;
  for (int k = 0; k < N; k++) {
    auto a = Clock::now();
    if (ffd_sample_create(e, gray.data(), W, H, W, &s) != FFD_OK) return 4;
    auto b = Clock::now();
    if (ffd_sample_eval_grid(s, FFD_FOREST_FFD, 0, 0, 3, nx, ny, trees.data(), 20, leaves.data()) != FFD_OK) return 5;
    auto c = Clock::now();
    t_create.push_back(us(a, b));
    t_first.push_back(us(b, c));
    for (int r = 0; r < 3; r++) {
      auto p = Clock::now();
      ffd_sample_eval_grid(s, FFD_FOREST_FFD, 0, 0, 3, nx, ny, trees.data(), 20, leaves.data());
      t_warm.push_back(us(p, Clock::now()));
    }
    ffd_sample_destroy(s);
  }
  std::printf("{\"sync_us\": %.2f, \"sample_create_us\": %.2f, \"first_grid_us\": %.2f, \"warm_grid_us\": %.2f, \"calls\": %d}\n",
              median(t_sync), median(t_create), median(t_first), median(t_warm), N);
  ffd_engine_destroy(e);
  return 0;
}
