#include "gguf.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <stdexcept>

#include "../common.h"

namespace lfk {

namespace {

enum VT : uint32_t { U8 = 0, I8, U16, I16, U32, I32, F32, BOOL, STR, ARR, U64, I64, F64 };

// Every length read from the file is checked against the bytes that remain before it
// is used (pointer arithmetic with an unchecked 64-bit length is undefined behaviour and
// could wrap past `end`; found by the ASan/UBSan mutation test, tests/test_sanitizers.py).
struct Cursor {
  const uint8_t* p;
  const uint8_t* end;
  size_t left() const { return (size_t)(end - p); }
  template <class T>
  T rd() {
    if (left() < sizeof(T)) throw std::runtime_error("gguf: truncated file");
    T v;
    std::memcpy(&v, p, sizeof(T));
    p += sizeof(T);
    return v;
  }
  std::string str() {
    const uint64_t n = rd<uint64_t>();
    if (n > left()) throw std::runtime_error("gguf: truncated string");
    std::string s(reinterpret_cast<const char*>(p), n);
    p += n;
    return s;
  }
  // an array of n elements of at least `min_bytes` each must fit in what is left
  // (bounds the reserve() below: a corrupt count cannot allocate gigabytes)
  void need(uint64_t n, size_t min_bytes) const {
    if (n > left() / min_bytes) throw std::runtime_error("gguf: array length exceeds the file");
  }
};

int64_t read_int(Cursor& c, uint32_t t) {
  switch (t) {
    case U8: return c.rd<uint8_t>();
    case I8: return c.rd<int8_t>();
    case U16: return c.rd<uint16_t>();
    case I16: return c.rd<int16_t>();
    case U32: return c.rd<uint32_t>();
    case I32: return c.rd<int32_t>();
    case U64: return (int64_t)c.rd<uint64_t>();
    case I64: return c.rd<int64_t>();
    case BOOL: return c.rd<uint8_t>();
  }
  throw std::runtime_error("gguf: not an int type");
}

GGUFValue read_value(Cursor& c, uint32_t t) {
  GGUFValue v;
  switch (t) {
    case F32: v.kind = GGUFValue::FLOAT; v.f = c.rd<float>(); break;
    case F64: v.kind = GGUFValue::FLOAT; v.f = c.rd<double>(); break;
    case BOOL: v.kind = GGUFValue::BOOL; v.b = c.rd<uint8_t>() != 0; v.i = v.b; break;
    case STR: v.kind = GGUFValue::STRING; v.s = c.str(); break;
    case ARR: {
      uint32_t et = c.rd<uint32_t>();
      uint64_t n = c.rd<uint64_t>();
      static const size_t kMinBytes[] = {1, 1, 2, 2, 4, 4, 4, 1, 8, 12, 8, 8, 8};
      if (et > F64) throw std::runtime_error("gguf: bad array element type");
      c.need(n, kMinBytes[et]);
      if (et == STR) {
        v.kind = GGUFValue::ARR_STRING;
        v.as.reserve(n);
        for (uint64_t i = 0; i < n; ++i) v.as.push_back(c.str());
      } else if (et == F32 || et == F64) {
        v.kind = GGUFValue::ARR_FLOAT;
        v.af.reserve(n);
        for (uint64_t i = 0; i < n; ++i) v.af.push_back(et == F32 ? c.rd<float>() : c.rd<double>());
      } else if (et == ARR) {
        throw std::runtime_error("gguf: nested arrays are not supported");
      } else {
        v.kind = et == BOOL ? GGUFValue::ARR_BOOL : GGUFValue::ARR_INT;
        v.ai.reserve(n);
        for (uint64_t i = 0; i < n; ++i) v.ai.push_back(read_int(c, et));
      }
      break;
    }
    default: v.kind = GGUFValue::INT; v.i = read_int(c, t); break;
  }
  return v;
}

}  // namespace

GGUFFile::GGUFFile(const std::string& path) : path_(path) {
  fd_ = ::open(path.c_str(), O_RDONLY);
  if (fd_ < 0) throw std::runtime_error("gguf: cannot open " + path);
  struct stat st;
  if (fstat(fd_, &st) != 0) {
    ::close(fd_);
    throw std::runtime_error("gguf: stat failed");
  }
  size_ = (size_t)st.st_size;
  void* m = mmap(nullptr, size_, PROT_READ, MAP_SHARED, fd_, 0);
  if (m == MAP_FAILED) {
    ::close(fd_);
    throw std::runtime_error("gguf: mmap failed");
  }
  base_ = static_cast<const uint8_t*>(m);
  // a constructor that throws never runs the destructor: release the mapping and the
  // fd here on every rejected file (bad magic, truncation, bounds, alignment)
  try {
    parse();
  } catch (...) {
    munmap(const_cast<uint8_t*>(base_), size_);
    ::close(fd_);
    base_ = nullptr;
    fd_ = -1;
    throw;
  }
}

void GGUFFile::parse() {
  Cursor c{base_, base_ + size_};
  if (c.rd<uint32_t>() != 0x46554747u) throw std::runtime_error("gguf: bad magic in " + path_);
  version_ = c.rd<uint32_t>();
  if (version_ < 2 || version_ > 3) throw std::runtime_error("gguf: unsupported version");
  uint64_t n_tensors = c.rd<uint64_t>();
  uint64_t n_kv = c.rd<uint64_t>();
  for (uint64_t i = 0; i < n_kv; ++i) {
    std::string key = c.str();
    uint32_t t = c.rd<uint32_t>();
    kv_[key] = read_value(c, t);
  }
  std::vector<std::pair<GGUFTensor, uint64_t>> infos;
  for (uint64_t i = 0; i < n_tensors; ++i) {
    GGUFTensor t;
    t.name = c.str();
    uint32_t nd = c.rd<uint32_t>();
    if (nd == 0 || nd > 4) throw std::runtime_error("gguf: tensor " + t.name + " has " + std::to_string(nd) + " dims");
    uint64_t count = 1;
    for (uint32_t d = 0; d < nd; ++d) {
      const uint64_t ne = c.rd<uint64_t>();
      // each dim and the element count stay far below 2^63 (n_elements() is int64)
      if (ne > (1ull << 40) || (ne && count > (1ull << 50) / ne))
        throw std::runtime_error("gguf: tensor " + t.name + " has an implausible shape");
      count *= ne;
      t.ne.push_back((int64_t)ne);
    }
    t.type = (int)c.rd<uint32_t>();
    uint64_t off = c.rd<uint64_t>();
    infos.push_back({t, off});
  }
  const int64_t align_i = get_int("general.alignment", 32);
  if (align_i <= 0 || align_i > (1 << 20) || (align_i & (align_i - 1)))
    throw std::runtime_error("gguf: general.alignment must be a power of two");
  const uint64_t align = (uint64_t)align_i;
  uint64_t pos = (uint64_t)(c.p - base_);
  uint64_t data_off = (pos + align - 1) / align * align;
  for (auto& [t, off] : infos) {
    const TypeInfo ti = type_info(t.type);
    const int64_t n = t.n_elements();
    if (t.ne[0] % ti.block) throw std::runtime_error("gguf: tensor " + t.name + " rows are not whole blocks");
    t.nbytes = (uint64_t)(n / ti.block) * ti.bytes;
    if (off > size_ || data_off > size_ - off || t.nbytes > size_ - data_off - off)
      throw std::runtime_error("gguf: tensor " + t.name + " out of bounds");
    t.offset = data_off + off;
    index_[t.name] = tensors_.size();
    tensors_.push_back(t);
  }
}

GGUFFile::~GGUFFile() {
  if (base_) munmap(const_cast<uint8_t*>(base_), size_);
  if (fd_ >= 0) ::close(fd_);
}

const GGUFTensor* GGUFFile::find(const std::string& name) const {
  auto it = index_.find(name);
  return it == index_.end() ? nullptr : &tensors_[it->second];
}

int64_t GGUFFile::get_int(const std::string& key, int64_t dflt) const {
  auto it = kv_.find(key);
  if (it == kv_.end()) return dflt;
  if (it->second.kind == GGUFValue::INT || it->second.kind == GGUFValue::BOOL) return it->second.i;
  if (it->second.kind == GGUFValue::FLOAT) return (int64_t)it->second.f;
  return dflt;
}

double GGUFFile::get_float(const std::string& key, double dflt) const {
  auto it = kv_.find(key);
  if (it == kv_.end()) return dflt;
  if (it->second.kind == GGUFValue::FLOAT) return it->second.f;
  if (it->second.kind == GGUFValue::INT) return (double)it->second.i;
  return dflt;
}

std::string GGUFFile::get_str(const std::string& key, const std::string& dflt) const {
  auto it = kv_.find(key);
  if (it == kv_.end() || it->second.kind != GGUFValue::STRING) return dflt;
  return it->second.s;
}

void GGUFFile::prefetch(const GGUFTensor& t) const {
  const size_t page = 4096;
  size_t start = t.offset / page * page;
  madvise(const_cast<uint8_t*>(base_) + start, t.offset + t.nbytes - start, MADV_WILLNEED);
}

}  // namespace lfk
