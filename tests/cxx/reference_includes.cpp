// reference_includes.cpp — a reference-style main against the C++ drop-in, with the reference's own include set
// (src/eval_ffd.cpp:11-13 and src/demo.cpp:11-16, minus trace.hpp / Viewer.hpp, the reference's logging and UI)
// and no #define: it uses every symbol of those headers that eval_ffd and demo use.  Built by
// tests/test_reference_includes.py with `g++ -Iinclude` so that the angle-bracket includes resolve to the forwarding
// headers of include/.
//
// modes:
//   cpu <annotations> <image.ppm> <config>          host-only pieces (no device needed), one "key value" per line
//   eval <config_headpose> <config_ffd> <cascade>     eval_ffd's main (src/eval_ffd.cpp:126-179): output/errors.txt
//   analyze <config_headpose> <config_ffd> <cascade> <image.ppm>
//                                                    demo's evalForest body (src/demo.cpp:102-154): analyzeImage
//   detect <cascade.xml> <image.ppm>                 the static FaceForest::detectFace with that classifier
//   train <config_ffd> <annotations> <n_images> <out_dir>
//                                                    demo's trainTree (src/demo.cpp:38-100) with the patches the
//                                                    engine's own trainer draws, against that trainer
#include <FaceForest.hpp>
#include <Constants.hpp>
#include <face_utils.hpp>
#include <Tree.hpp>
#include <ImageSample.hpp>
#include <MPSample.hpp>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <random>
#include <string>
#include <vector>

// eval_ffd.cpp:33-46
float getInterOccularDist(const FaceAnnotation& annotation) {
  cv::Point2f center_left, center_right;
  center_left.x = (annotation.parts[0].x + annotation.parts[1].x) / 2.0f;
  center_left.y = (annotation.parts[0].y + annotation.parts[1].y) / 2.0f;
  center_right.x = (annotation.parts[6].x + annotation.parts[7].x) / 2.0f;
  center_right.y = (annotation.parts[6].y + annotation.parts[7].y) / 2.0f;
  return cv::norm(center_left - center_right);
}

// eval_ffd.cpp:58-124 (progress display, TRACE and the viewer left out)
void evalForest(FaceForestOptions ff_options, std::vector<std::vector<FaceAnnotation> >& ann) {
  FaceForest ff(ff_options);
  std::vector<FaceAnnotation> annotations;
  for (unsigned int i = 0; i < ann.size(); i++) annotations.insert(annotations.end(), ann[i].begin(), ann[i].end());
  std::vector<std::vector<float> > errors;
  for (int i = 0; i < static_cast<int>(annotations.size()); ++i) {
    cv::Mat img = loadImage(ff_options.mp_forest_param.image_path, annotations[i].url);
    if (img.empty()) {
      std::cerr << "Could not load: " << annotations[i].url << std::endl;
      continue;
    }
    Face face;
    ff.analyzeFace(img, annotations[i].bbox, face);
    std::vector<float> err;
    float inter_occular_dist = getInterOccularDist(annotations[i]);
    for (int j = 0; j < (int)face.ffd_cordinates.size(); j++) {
      float d = cv::norm(annotations[i].parts[j] - face.ffd_cordinates[j]);
      err.push_back(d / inter_occular_dist);
    }
    errors.push_back(err);
  }
  std::ofstream ofs;
  std::string path = "output/errors.txt";
  ofs.open(path.c_str(), std::ios::out);
  for (size_t i = 0; i < errors.size(); i++) {
    for (size_t j = 0; j < errors[i].size(); j++) ofs << errors[i][j] << " ";
    ofs << std::endl;
  }
}

static bool options_from(const char* hp_cfg, const char* ffd_cfg, const char* cascade, FaceForestOptions& ff_options) {
  ForestParam hp_param, mp_param;
  if (!loadConfigFile(hp_cfg, hp_param)) return false;
  if (!loadConfigFile(ffd_cfg, mp_param)) return false;
  ff_options.fd_option.path_face_cascade = cascade;
  ff_options.hp_forest_param = hp_param;
  ff_options.mp_forest_param = mp_param;
  return true;
}

// eval_ffd.cpp:126-179
static int eval_main(const char* hp_cfg, const char* ffd_cfg, const char* face_cascade) {
  ForestParam hp_param, mp_param;
  if (!loadConfigFile(hp_cfg, hp_param)) return EXIT_FAILURE;
  if (!loadConfigFile(ffd_cfg, mp_param)) return EXIT_FAILURE;
  std::vector<FaceAnnotation> annotations;
  if (!loadAnnotations(mp_param.image_path, annotations)) return EXIT_FAILURE;
  std::vector<std::vector<FaceAnnotation> > ann(NUM_HEADPOSE_CLASSES);
  for (unsigned int i = 0; i < annotations.size(); i++) ann[annotations[i].pose + 2].push_back(annotations[i]);
  std::vector<std::vector<FaceAnnotation> > test_ann(NUM_HEADPOSE_CLASSES);
  for (unsigned int i = 0; i < ann.size(); i++) {
    int num_train_imgs = static_cast<int>(ann[i].size() * TRAIN_IMAGES_PERCENTAGE);
    test_ann[i].insert(test_ann[i].begin(), ann[i].begin() + num_train_imgs, ann[i].end());
  }
  FaceForestOptions ff_options;
  ff_options.fd_option.path_face_cascade = face_cascade;
  ff_options.hp_forest_param = hp_param;
  ff_options.mp_forest_param = mp_param;
  evalForest(ff_options, test_ann);
  return EXIT_SUCCESS;
}

// demo.cpp:102-154 (viewer left out): detect and analyze every face of an image
static int analyze_main(const char* hp_cfg, const char* ffd_cfg, const char* cascade, const char* image) {
  FaceForestOptions ff_options;
  if (!options_from(hp_cfg, ffd_cfg, cascade, ff_options)) return EXIT_FAILURE;
  std::unique_ptr<ImageSample> kept;  // made under the FaceForest below and kept past its end
  {
    FaceForest ff(ff_options);
    if (!ff.is_initialized()) return 3;
    cv::Mat img = loadImage(image, std::string(image).substr(std::string(image).rfind('/') + 1));
    if (img.empty()) return 4;
    std::vector<Face> faces;
    ff.analyzeImage(img, faces);
    for (const Face& f : faces) {
      std::printf("face %d %d %d %d %.9g", f.bbox.x, f.bbox.y, f.bbox.width, f.bbox.height, f.headpose);
      for (const cv::Point& p : f.ffd_cordinates) std::printf(" %d %d", p.x, p.y);
      std::printf("\n");
    }
    cv::Mat gray(64, 64, CV_8UC1);
    for (int y = 0; y < 64; y++)
      for (int x = 0; x < 64; x++) gray.data[(size_t)y * gray.step + x] = img.data[(size_t)y * img.step + 3 * x];
    kept.reset(new ImageSample(gray, std::vector<int>{0, 1, 2}, true));
    (void)kept->channels();
  }
  // the engine is gone: it freed the sample's planes, the sample's calls fail, its destructor frees host state only
  int threw = 0;
  try {
    ImageSample copy = *kept;
    std::vector<uint32_t> ch(38 * 65 * 65);
    if (ffd_sample_channels(copy.handle(), ch.data()) != FFD_OK) threw = 1;
  } catch (const std::exception&) {
    threw = 1;
  }
  kept.reset();
  std::printf("orphaned_sample_fails %d\n", threw);
  return EXIT_SUCCESS;
}

// FaceForest::detectFace(img, face_cascade, fd_option, boxes) with the caller's classifier (FaceForest.hpp:125-132)
static int detect_main(const char* xml, const char* image) {
  cv::CascadeClassifier face_cascade;
  if (!face_cascade.load(xml)) {
    std::printf("load failed\n");
    return 5;
  }
  cv::Mat img = loadImage(image, std::string(image).substr(std::string(image).rfind('/') + 1));
  if (img.empty()) return 4;
  FaceDetectionOption fd_option;
  std::vector<cv::Rect> faces_bboxes;
  FaceForest::detectFace(img, face_cascade, fd_option, faces_bboxes);
  for (const cv::Rect& r : faces_bboxes) std::printf("box %d %d %d %d\n", r.x, r.y, r.width, r.height);
  std::printf("n %zu\n", faces_bboxes.size());
  return EXIT_SUCCESS;
}

// demo.cpp:38-100's trainTree over the first n annotated images: gray, scaled to face_size, enlarged face ROI,
// ImageSample, MPSamples at the patches, Tree<MPSample>(samples, param, &rng, path).  The patches are the ones the
// engine's own trainer draws from tree_seed (ffd_train_mp_tree, whose trees are pinned to the oracle's), so the two
// trees must be the same archive byte for byte.
static int train_main(const char* ffd_cfg, const char* ann_path, int n_images, const char* out_dir) {
  ForestParam mp_param;
  if (!loadConfigFile(ffd_cfg, mp_param)) return EXIT_FAILURE;
  std::vector<FaceAnnotation> annotations;
  if (!loadAnnotations(ann_path, annotations)) return EXIT_FAILURE;
  mp_param.npatches = 60;
  mp_param.ntests = 200;
  mp_param.max_depth = 8;
  std::vector<cv::Mat> rois;
  std::vector<std::vector<int32_t> > parts;
  for (int i = 0; i < n_images && i < (int)annotations.size(); i++) {
    cv::Mat img = loadImage(ann_path, annotations[i].url);
    if (img.empty()) return 4;
    // gray (BT.601 fixed point as cv::cvtColor) and a nearest-neighbour scale to face_size: any deterministic
    // image does here, both trees see the same pixels
    float scale = static_cast<float>(mp_param.face_size) / static_cast<float>(annotations[i].bbox.width);
    cv::Mat img_scaled(static_cast<int>(img.rows * scale), static_cast<int>(img.cols * scale), CV_8UC1);
    for (int y = 0; y < img_scaled.rows; y++)
      for (int x = 0; x < img_scaled.cols; x++) {
        const uint8_t* p = img.data + (size_t)std::min(img.rows - 1, (int)(y / scale)) * img.step +
                           3 * std::min(img.cols - 1, (int)(x / scale));
        img_scaled.data[(size_t)y * img_scaled.step + x] = (uint8_t)((p[0] * 1868 + p[1] * 9617 + p[2] * 4899 + 8192) >> 14);
      }
    annotations[i].bbox.x *= scale;
    annotations[i].bbox.y *= scale;
    annotations[i].bbox.width *= scale;
    annotations[i].bbox.height *= scale;
    for (unsigned int j = 0; j < annotations[i].parts.size(); j++) annotations[i].parts[j] *= scale;
    cv::Rect enlarge_bbox;
    enlargeFace(img_scaled, enlarge_bbox, annotations[i]);
    rois.push_back(img_scaled(enlarge_bbox).clone());
    std::vector<int32_t> pv;
    for (const cv::Point& p : annotations[i].parts) pv.insert(pv.end(), {p.x, p.y});
    parts.push_back(pv);
  }
  // the engine's trainer (ffd_train_mp_tree: npatches draws per image from tree_seed)
  std::vector<ffd_train_image> ti(rois.size());
  for (size_t k = 0; k < rois.size(); k++)
    ti[k] = ffd_train_image{rois[k].data, rois[k].cols, rois[k].rows, (int32_t)rois[k].step, parts[k].data()};
  ffd_train_param tp;
  ffd_train_param_init(&tp);
  tp.max_depth = mp_param.max_depth; tp.min_patches = mp_param.min_patches; tp.ntests = mp_param.ntests;
  tp.npatches = mp_param.npatches; tp.face_size = mp_param.face_size; tp.patch_size_ratio = mp_param.patch_size_ratio;
  tp.ntrees = mp_param.ntrees; tp.nimages = mp_param.nimages;  // (the archive records the ForestParam, as Tree::save)
  tp.tree_seed = 100;
  tp.split_seed = (uint32_t)std::strtoul(std::getenv("FFD_SPLIT_SEED") ? std::getenv("FFD_SPLIT_SEED") : "7", nullptr, 10);
  char tree_path[512];  // (the path the shim's Tree below saves to: the archive records it)
  std::snprintf(tree_path, sizeof tree_path, "%s/tree_%03d.txt", out_dir, 98);
  tp.tree_path = mp_param.tree_path.c_str();
  tp.image_path = mp_param.image_path.c_str();
  tp.save_path = tree_path;
  ffd_trained_tree* ref = nullptr;
  if (ffd_train_mp_tree(&tp, ti.data(), (int32_t)ti.size(), &ref) != FFD_OK) {
    std::printf("train failed: %s\n", ffd_train_last_error());
    return 6;
  }
  const int64_t n = ffd_trained_tree_num_samples(ref);
  std::vector<int32_t> xy(3 * n);
  ffd_trained_tree_arrays(ref, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, xy.data());
  // demo.cpp:86-96: one ImageSample per ROI, an MPSample per patch
  std::vector<ImageSample*> images;
  for (size_t k = 0; k < rois.size(); k++) images.push_back(new ImageSample(rois[k], mp_param.features, false));
  std::vector<MPSample*> mp_samples;
  mp_samples.reserve(mp_param.nimages * mp_param.npatches);
  const int patch_size = mp_param.getPatchSize();
  for (int64_t j = 0; j < n; j++) {
    const int k = xy[3 * j];
    cv::Rect bbox = cv::Rect(xy[3 * j + 1], xy[3 * j + 2], patch_size, patch_size);
    std::vector<cv::Point> pts;
    for (int q = 0; q < 10; q++) pts.push_back(cv::Point(parts[k][2 * q], parts[k][2 * q + 1]));
    mp_samples.push_back(new MPSample(images[k], bbox, pts, mp_param.face_size, true));
  }
  std::mt19937 rng(100);
  char tree_path2[512];
  std::snprintf(tree_path2, sizeof tree_path2, "%s/tree_%03d.txt", out_dir, 98);
  mp_param.tree_path = tp.tree_path;
  Tree<MPSample>* tree = new Tree<MPSample>(mp_samples, mp_param, &rng, tree_path2);
  int64_t sa = 0, sb = 0;
  ffd_trained_tree_archive(ref, nullptr, 0, &sa);
  ffd_trained_tree_archive(tree->trained.get(), nullptr, 0, &sb);
  std::string a((size_t)sa, '\0'), b((size_t)sb, '\0');
  ffd_trained_tree_archive(ref, &a[0], sa, &sa);
  ffd_trained_tree_archive(tree->trained.get(), &b[0], sb, &sb);
  std::printf("samples %lld nodes %lld nodes_shim %lld same_archive %d\n", (long long)n, (long long)ffd_trained_tree_num_nodes(ref),
              (long long)ffd_trained_tree_num_nodes(tree->trained.get()), a == b ? 1 : 0);
  std::ifstream saved(tree_path2, std::ios::binary);
  std::string file((std::istreambuf_iterator<char>(saved)), std::istreambuf_iterator<char>());
  std::printf("saved_equal %d\n", file == b ? 1 : 0);
  ffd_trained_tree_free(ref);
  delete tree;
  for (MPSample* s : mp_samples) delete s;
  for (ImageSample* s : images) delete s;
  return EXIT_SUCCESS;
}

// host-only pieces: the readers, the split, loadImage, enlargeFace, the geometry helpers and the constants
static int cpu_main(const char* ann_path, const char* ppm, const char* cfg) {
  ForestParam p;
  const bool cfg_ok = loadConfigFile(cfg, p);
  std::printf("config %d %s %d %d %d\n", cfg_ok ? 1 : 0, p.tree_path.c_str(), p.ntrees, p.face_size, p.getPatchSize());
  std::vector<FaceAnnotation> annotations;
  const bool ann_ok = loadAnnotations(ann_path, annotations);
  std::printf("annotations %d %zu\n", ann_ok ? 1 : 0, annotations.size());
  std::vector<std::vector<FaceAnnotation> > ann(NUM_HEADPOSE_CLASSES);
  for (unsigned int i = 0; i < annotations.size(); i++) ann[annotations[i].pose + 2].push_back(annotations[i]);
  std::printf("test_split");
  for (unsigned int i = 0; i < ann.size(); i++) {
    int num_train_imgs = static_cast<int>(ann[i].size() * TRAIN_IMAGES_PERCENTAGE);
    for (size_t j = num_train_imgs; j < ann[i].size(); j++) std::printf(" %s", ann[i][j].url.c_str());
  }
  std::printf("\n");
  cv::Mat img = loadImage(ppm, std::string(ppm).substr(std::string(ppm).rfind('/') + 1));
  std::printf("image %d %d %d %d %d %d\n", img.empty() ? 0 : 1, img.rows, img.cols, img.channels(),
              img.empty() ? -1 : img.data[0], img.empty() ? -1 : img.data[img.step * (img.rows - 1) + 3 * img.cols - 1]);
  FaceAnnotation a = annotations.at(0);
  cv::Rect enlarge_bbox;
  enlargeFace(img, enlarge_bbox, a);
  std::printf("enlarge %d %d %d %d %d %d\n", enlarge_bbox.x, enlarge_bbox.y, enlarge_bbox.width, enlarge_bbox.height,
              a.parts[0].x, a.parts[0].y);
  cv::Mat roi = img(enlarge_bbox);
  std::printf("roi %d %d %d\n", roi.rows, roi.cols, roi.data[0]);
  std::printf("iod %.9g\n", getInterOccularDist(annotations.at(0)));
  cv::Rect r = intersect(cv::Rect(-5, -5, 20, 20), cv::Rect(0, 0, 10, 10));
  std::printf("intersect %d %d %d %d\n", r.x, r.y, r.width, r.height);
  std::printf("area %.9g\n", areaUnderCurve(-1.f, 1.f, 0.0, 1.0));
  std::printf("constants %.9g %d %.9g %.9g\n", TRAIN_IMAGES_PERCENTAGE, NUM_HEADPOSE_CLASSES, NORM_HEADPOSE_VARIANCE_FACTOR,
              PATCH_CLOSE_TO_FEATURE);
  cv::Point q(7, 9);
  q *= 0.5f;  // cvRound: 3.5 -> 4, 4.5 -> 4
  std::printf("scaled %d %d\n", q.x, q.y);
  FaceForestOptions o;
  FaceForest ff(o);  // no tree paths, no model: not initialised, as the reference's ctor on a missing cascade
  std::printf("initialized %d\n", ff.is_initialized() ? 1 : 0);
  return EXIT_SUCCESS;
}

// FaceForest(FaceForestOptions) over the reference's tree directories with the given cascade path: the reference's
// constructor returns uninitialised when the cascade does not load (FaceForest.cpp:23-27)
static int init_main(const char* hp_cfg, const char* ffd_cfg, const char* cascade) {
  FaceForestOptions ff_options;
  if (!options_from(hp_cfg, ffd_cfg, cascade, ff_options)) return EXIT_FAILURE;
  FaceForest ff(ff_options);
  std::printf("initialized %d\n", ff.is_initialized() ? 1 : 0);
  return EXIT_SUCCESS;
}

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "";
  try {
    if (mode == "cpu" && argc == 5) return cpu_main(argv[2], argv[3], argv[4]);
    if (mode == "eval" && argc == 5) return eval_main(argv[2], argv[3], argv[4]);
    if (mode == "analyze" && argc == 6) return analyze_main(argv[2], argv[3], argv[4], argv[5]);
    if (mode == "detect" && argc == 4) return detect_main(argv[2], argv[3]);
    if (mode == "init" && argc == 5) return init_main(argv[2], argv[3], argv[4]);
    if (mode == "train" && argc == 6) return train_main(argv[2], argv[3], std::atoi(argv[4]), argv[5]);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "exception: %s\n", e.what());
    return 9;
  }
  std::fprintf(stderr, "usage: see the header of tests/cxx/reference_includes.cpp\n");
  return 2;
}
