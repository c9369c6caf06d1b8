// Which engine a reference call without one uses (VERDICT r5 "next" #6): ImageSample(img, features, ...),
// MeanShift::shift / mode and Forest<S>::load take no engine in the reference (src/ImageSample.cpp:11-20,
// include/MeanShift.hpp:41-76, include/Forest.hpp:103-129).  With one FaceForest alive they use its engine; with
// several alive they fail with a clear error instead of binding to the last-constructed one.
//
//   engine_choice cpu          the registry logic with two placeholder engines (no device, no call into libffd)
//   engine_choice gpu MODEL    two real FaceForests on device 0
#include <FaceForest.hpp>

using namespace ffd;

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

static int failures = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::printf("FAIL line %d: %s\n", __LINE__, #c);             \
      failures++;                                                  \
    }                                                              \
  } while (0)

// runs f and returns the runtime_error text ("" when nothing was thrown)
template <class F>
static std::string error_of(F&& f) {
  try {
    f();
  } catch (const std::runtime_error& e) {
    return e.what();
  }
  return "";
}

static std::vector<uint8_t> face_pixels(int w, int h) {
  std::vector<uint8_t> g((size_t)w * h);
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) g[(size_t)y * w + x] = (uint8_t)((x * 7 + y * 13 + (x * y) % 23) & 255);
  return g;
}

static std::vector<Vote> some_votes() {
  std::vector<Vote> v;
  for (int i = 0; i < 40; i++) {
    Vote a;
    a.pos = Point(60 + (i % 7), 50 + (i % 5));
    a.weight = 1.f + 0.01f * i;
    a.check = true;
    v.push_back(a);
  }
  return v;
}

static int run_cpu() {
  const std::vector<uint8_t> g = face_pixels(125, 125);
  // no FaceForest: an ImageSample is made without an engine (the training-program case, demo.cpp:86-96)
  CHECK(detail::live_engines() == 0);
  CHECK(error_of([&] { ImageSample s(g.data(), 125, 125, 125); }).empty());
  CHECK(error_of([&] { float m[2]; MeanShift::mode(some_votes(), m); }).find("no FaceForest engine") != std::string::npos);
  ImageSample late(g.data(), 125, 125, 125);
  // two placeholder engines with the same tree directories
  ffd_engine* e1 = reinterpret_cast<ffd_engine*>(0x1000);
  ffd_engine* e2 = reinterpret_cast<ffd_engine*>(0x2000);
  detail::ForestDirs d1, d2;
  d1.engine = e1;
  d2.engine = e2;
  d1.hp_dir = d2.hp_dir = "/trees/headpose";
  d1.mp_dirs = d2.mp_dirs = {"/trees/ffd/0", "/trees/ffd/1"};
  detail::register_engine(d1);
  CHECK(detail::default_engine("t") == e1);  // one alive: its engine, as the reference's signatures need
  detail::register_engine(d2);
  const std::string es = error_of([&] { ImageSample s(g.data(), 125, 125, 125); });
  CHECK(es.find("ImageSample") != std::string::npos && es.find("2 FaceForests are alive") != std::string::npos);
  const std::string em = error_of([&] { float m[2]; MeanShift::mode(some_votes(), m); });
  CHECK(em.find("MeanShift") != std::string::npos && em.find("ambiguous") != std::string::npos);
  const std::string eh = error_of([&] { Point p; MeanShift::shift(some_votes(), p, 7, 10, 0.05f); });
  CHECK(eh.find("ambiguous") != std::string::npos);
  // an ImageSample made while no engine was alive binds on first use: ambiguous now
  CHECK(error_of([&] { late.handle(); }).find("ambiguous") != std::string::npos);
  // Forest::load: both engines hold the directory -> refused; with the engine named -> that engine's trees
  Forest<MPSample> f;
  ForestParam fp;
  fp.ntrees = 3;
  CHECK(!f.load("/trees/ffd/1", fp));
  CHECK(f.load("/trees/ffd/1", fp, -1, e2) && f.engine() == e2 && f.numberOfTrees() == 3);
  // one left: the default is the survivor
  detail::unregister_engine(e2);
  CHECK(detail::default_engine("t") == e1);
  Forest<MPSample> f1;
  CHECK(f1.load("/trees/ffd/0", fp) && f1.engine() == e1);
  detail::unregister_engine(e1);
  CHECK(detail::live_engines() == 0);
  std::printf("cpu checks done, failures %d\n", failures);
  return failures ? 1 : 0;
}

static int run_gpu(const char* model) {
  const std::vector<uint8_t> g = face_pixels(125, 125);
  FaceForestOptions opt;
  opt.model_path = model;
  std::vector<Vote> votes = some_votes();
  float want[2];
  {
    FaceForest a(opt);
    CHECK(a.is_initialized());
    // one FaceForest: the reference's engine-less calls work and use it
    ImageSample s(g.data(), 125, 125, 125);
    CHECK(s.engine() == a.engine());
    MeanShift::mode(votes, want);
    {
      FaceForest b(opt);
      CHECK(b.is_initialized() && b.engine() != a.engine());
      CHECK(error_of([&] { ImageSample t(g.data(), 125, 125, 125); }).find("ambiguous") != std::string::npos);
      CHECK(error_of([&] { float m[2]; MeanShift::mode(votes, m); }).find("ambiguous") != std::string::npos);
      // named engines work, and each gives the same mode
      ImageSample tb(g.data(), 125, 125, 125, {0, 1, 2}, true, b.engine());
      CHECK(tb.engine() == b.engine());
      float mb[2];
      MeanShift::mode(votes, mb, 7, 10, 0.05f, b.engine());
      CHECK(std::memcmp(mb, want, sizeof(mb)) == 0);
      // the sample bound to `a` before `b` existed keeps `a`
      CHECK(s.engine() == a.engine());
    }
    // `b` is gone: the default is `a` again
    ImageSample u(g.data(), 125, 125, 125);
    CHECK(u.engine() == a.engine());
    float m2[2];
    MeanShift::mode(votes, m2);
    CHECK(std::memcmp(m2, want, sizeof(m2)) == 0);
  }
  std::printf("gpu checks done, failures %d\n", failures);
  return failures ? 1 : 0;
}

int main(int argc, char** argv) {
  if (argc >= 2 && std::string(argv[1]) == "cpu") return run_cpu();
  if (argc >= 3 && std::string(argv[1]) == "gpu") return run_gpu(argv[2]);
  std::fprintf(stderr, "usage: %s cpu | gpu MODEL\n", argv[0]);
  return 2;
}
