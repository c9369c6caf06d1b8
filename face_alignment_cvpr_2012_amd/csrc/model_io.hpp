// model_io.hpp — reader/writer for the FFDMODEL container (include/ffd_model_format.h).
//
// Product-side replacement of the reference loader Forest<S>::load / load_tree
// (/root/reference/include/Forest.hpp:103-153): the archive parse happens once
// offline (ffd_convert.cpp); at run time the engine maps named arrays.
#pragma once

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "ffd_model_format.h"

namespace ffd {

struct ModelArray {
  std::string dtype;
  std::vector<uint64_t> shape;
  std::vector<uint8_t> bytes;

  uint64_t count() const {
    uint64_t n = 1;
    for (auto s : shape) n *= s;
    return n;
  }
  template <typename T> const T* as() const { return reinterpret_cast<const T*>(bytes.data()); }
  template <typename T> T* as() { return reinterpret_cast<T*>(bytes.data()); }
};

class ModelFile {
 public:
  std::map<std::string, ModelArray> arrays;

  bool has(const std::string& n) const { return arrays.count(n) != 0; }

  const ModelArray& get(const std::string& n) const {
    auto it = arrays.find(n);
    if (it == arrays.end()) throw std::runtime_error("model array missing: " + n);
    return it->second;
  }

  template <typename T>
  void put(const std::string& name, const char* dtype, const std::vector<uint64_t>& shape,
           const std::vector<T>& data) {
    ModelArray a;
    a.dtype = dtype;
    a.shape = shape;
    uint64_t n = a.count();
    if (n != data.size()) throw std::runtime_error("shape/data mismatch for " + name);
    a.bytes.resize(n * sizeof(T));
    if (n) std::memcpy(a.bytes.data(), data.data(), n * sizeof(T));
    arrays[name] = std::move(a);
  }

  void save(const std::string& path) const {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot write " + path);
    std::vector<ffd_array_entry> ents;
    uint64_t off = 8 + 4 + 4 + arrays.size() * sizeof(ffd_array_entry);
    auto align = [](uint64_t v) { return (v + FFD_MODEL_ALIGN - 1) / FFD_MODEL_ALIGN * FFD_MODEL_ALIGN; };
    off = align(off);
    for (auto& kv : arrays) {
      ffd_array_entry e;
      std::memset(&e, 0, sizeof(e));
      if (kv.first.size() >= sizeof(e.name)) throw std::runtime_error("name too long");
      std::strncpy(e.name, kv.first.c_str(), sizeof(e.name) - 1);
      std::strncpy(e.dtype, kv.second.dtype.c_str(), sizeof(e.dtype) - 1);
      e.ndim = (uint32_t)kv.second.shape.size();
      for (size_t i = 0; i < kv.second.shape.size() && i < 4; i++) e.shape[i] = kv.second.shape[i];
      e.offset = off;
      e.nbytes = kv.second.bytes.size();
      off = align(off + e.nbytes);
      ents.push_back(e);
    }
    uint32_t ver = FFD_MODEL_VERSION, n = (uint32_t)ents.size();
    std::fwrite(FFD_MODEL_MAGIC, 1, 8, f);
    std::fwrite(&ver, 4, 1, f);
    std::fwrite(&n, 4, 1, f);
    std::fwrite(ents.data(), sizeof(ffd_array_entry), ents.size(), f);
    uint64_t pos = 16 + ents.size() * sizeof(ffd_array_entry);
    static const uint8_t zeros[FFD_MODEL_ALIGN] = {0};
    size_t i = 0;
    for (auto& kv : arrays) {
      const auto& e = ents[i++];
      while (pos < e.offset) {
        size_t k = (size_t)std::min<uint64_t>(e.offset - pos, FFD_MODEL_ALIGN);
        std::fwrite(zeros, 1, k, f);
        pos += k;
      }
      if (e.nbytes) std::fwrite(kv.second.bytes.data(), 1, e.nbytes, f);
      pos += e.nbytes;
    }
    if (std::fclose(f) != 0) throw std::runtime_error("write failed: " + path);
  }

  // only: load just the arrays whose name contains this substring (empty: all of them)
  void load(const std::string& path, const std::string& only = std::string()) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) throw std::runtime_error("cannot open model file " + path);
    char magic[8];
    uint32_t ver = 0, n = 0;
    if (std::fread(magic, 1, 8, f) != 8 || std::memcmp(magic, FFD_MODEL_MAGIC, 8) != 0) {
      std::fclose(f);
      throw std::runtime_error("not an FFDMODEL file: " + path);
    }
    if (std::fread(&ver, 4, 1, f) != 1 || ver != FFD_MODEL_VERSION || std::fread(&n, 4, 1, f) != 1) {
      std::fclose(f);
      throw std::runtime_error("unsupported FFDMODEL version in " + path);
    }
    std::vector<ffd_array_entry> ents(n);
    if (n && std::fread(ents.data(), sizeof(ffd_array_entry), n, f) != n) {
      std::fclose(f);
      throw std::runtime_error("truncated header in " + path);
    }
    arrays.clear();
    for (auto& e : ents) {
      if (!only.empty() && std::string(e.name, strnlen(e.name, sizeof(e.name))).find(only) == std::string::npos) continue;
      ModelArray a;
      a.dtype = std::string(e.dtype, strnlen(e.dtype, sizeof(e.dtype)));
      for (uint32_t i = 0; i < e.ndim && i < 4; i++) a.shape.push_back(e.shape[i]);
      a.bytes.resize(e.nbytes);
      if (std::fseek(f, (long)e.offset, SEEK_SET) != 0 ||
          (e.nbytes && std::fread(a.bytes.data(), 1, e.nbytes, f) != e.nbytes)) {
        std::fclose(f);
        throw std::runtime_error("truncated array in " + path);
      }
      arrays[std::string(e.name, strnlen(e.name, sizeof(e.name)))] = std::move(a);
    }
    std::fclose(f);
  }
};

}  // namespace ffd
