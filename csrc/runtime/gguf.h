// Native GGUF v2/v3 parser over a read-only mmap.
// Tensor payloads are never copied at parse time: `data(name)` is a pointer
// into the mapping, streamed to the GPU (after the planar repack) at load.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace lfk {

struct GGUFValue {
  enum Kind { NONE, INT, FLOAT, BOOL, STRING, ARR_INT, ARR_FLOAT, ARR_STRING, ARR_BOOL } kind = NONE;
  int64_t i = 0;
  double f = 0;
  bool b = false;
  std::string s;
  std::vector<int64_t> ai;
  std::vector<double> af;
  std::vector<std::string> as;
};

struct GGUFTensor {
  std::string name;
  int type = 0;
  std::vector<int64_t> ne;  // ggml order: ne[0] innermost
  uint64_t offset = 0;      // absolute file offset
  uint64_t nbytes = 0;
  int64_t n_elements() const {
    int64_t n = 1;
    for (auto d : ne) n *= d;
    return n;
  }
};

class GGUFFile {
 public:
  explicit GGUFFile(const std::string& path);
  ~GGUFFile();
  GGUFFile(const GGUFFile&) = delete;
  GGUFFile& operator=(const GGUFFile&) = delete;

  const std::map<std::string, GGUFValue>& metadata() const { return kv_; }
  const std::vector<GGUFTensor>& tensors() const { return tensors_; }
  const GGUFTensor* find(const std::string& name) const;
  const uint8_t* data(const GGUFTensor& t) const { return base_ + t.offset; }
  bool has(const std::string& key) const { return kv_.count(key) > 0; }
  int64_t get_int(const std::string& key, int64_t dflt) const;
  double get_float(const std::string& key, double dflt) const;
  std::string get_str(const std::string& key, const std::string& dflt) const;
  uint32_t version() const { return version_; }
  size_t file_size() const { return size_; }
  // advise the kernel to read ahead a tensor's pages (overlaps disk IO with the repack)
  void prefetch(const GGUFTensor& t) const;

 private:
  void parse();  // header, KV pairs and tensor infos of the mapped file (throws on malformed input)

  std::string path_;
  int fd_ = -1;
  const uint8_t* base_ = nullptr;
  size_t size_ = 0;
  uint32_t version_ = 0;
  std::map<std::string, GGUFValue> kv_;
  std::vector<GGUFTensor> tensors_;
  std::map<std::string, size_t> index_;
};

}  // namespace lfk
