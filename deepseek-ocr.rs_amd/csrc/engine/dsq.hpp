// DSQ snapshot container (crates/dsq/src/lib.rs): mmap + index + the reader's validation rules.
//   header  magic "DSQSNAP" (14), u32 version == 1 (15, 321-327), u32-length strings
//           candle_version / model_id / backend (328-330, 521-528), u32 default qdtype (331-332),
//           u32 block_size != 0 (333-338), u32 tensor_count (339)
//   record  string name, u32 out_dim, u32 in_dim, u32 q_dtype, u64 q_offset, u64 q_len,
//           u64 bias_offset, u64 bias_len (0: no bias), u32 bias_dtype (341-369)
//   checks  default qdtype quantised + block_size matching it (393-407); per record: non-empty
//           payload past the metadata, slices inside the file, in_dim % block == 0 for k-quants,
//           exact byte length for float records, no duplicate names (409-519, 225-233)
// Errors map to DSOCR_EINVAL (malformed / unsupported) and DSOCR_ENOENT (missing file).
#pragma once

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdint>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "../kernels/kernels.hpp"

namespace dsocr {

struct DsqRecord {
    std::string name;
    uint32_t out_dim = 0, in_dim = 0;
    int q_dtype = 0;
    uint64_t q_offset = 0, q_len = 0;
    bool has_bias = false;
    uint64_t bias_offset = 0, bias_len = 0;
    int bias_dtype = 0;
};

class DsqFile {
public:
    explicit DsqFile(const std::string& path) : path_(path) {
        fd_ = ::open(path.c_str(), O_RDONLY);
        if (fd_ < 0) throw std::runtime_error("ENOENT: cannot open snapshot " + path);
        struct stat st;
        if (fstat(fd_, &st) != 0) { ::close(fd_); throw std::runtime_error("ENOENT: cannot stat snapshot " + path); }
        size_ = (size_t)st.st_size;
        if (size_ == 0) { ::close(fd_); throw std::runtime_error("EINVAL: snapshot malformed: empty file " + path); }
        void* p = mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd_, 0);
        if (p == MAP_FAILED) { ::close(fd_); throw std::runtime_error("EINVAL: cannot map snapshot " + path); }
        data_ = static_cast<const uint8_t*>(p);
        try {
            parse();
        } catch (...) {
            munmap(const_cast<uint8_t*>(data_), size_);
            ::close(fd_);
            throw;
        }
    }
    ~DsqFile() {
        if (data_) munmap(const_cast<uint8_t*>(data_), size_);
        if (fd_ >= 0) ::close(fd_);
    }
    DsqFile(const DsqFile&) = delete;
    DsqFile& operator=(const DsqFile&) = delete;

    const DsqRecord* find(const std::string& name) const {
        auto it = index_.find(name);
        return it == index_.end() ? nullptr : &records_[it->second];
    }
    const std::vector<DsqRecord>& records() const { return records_; }
    const uint8_t* payload(const DsqRecord& r) const { return data_ + r.q_offset; }
    int default_qdtype() const { return default_qdtype_; }
    const std::string& model_id() const { return model_id_; }

    // bias values as f32 (U8 / U32 / I64 / F16 / F32 / F64 / BF16, lib.rs:137-168)
    std::vector<float> bias(const DsqRecord& r) const {
        std::vector<float> out;
        if (!r.has_bias) return out;
        const uint8_t* p = data_ + r.bias_offset;
        const size_t esz = r.bias_dtype == 0 ? 1 : (r.bias_dtype == 2 || r.bias_dtype == 5) ? 8
                                                 : (r.bias_dtype == 3 || r.bias_dtype == 6) ? 2 : 4;
        const size_t n = r.bias_len / esz;
        out.resize(n);
        for (size_t i = 0; i < n; ++i) {
            const uint8_t* q = p + i * esz;
            switch (r.bias_dtype) {
                case 0: out[i] = (float)q[0]; break;
                case 1: { uint32_t v; std::memcpy(&v, q, 4); out[i] = (float)v; break; }
                case 2: { int64_t v; std::memcpy(&v, q, 8); out[i] = (float)v; break; }
                case 3: { uint16_t v; std::memcpy(&v, q, 2); out[i] = half_to_f32(v); break; }
                case 4: std::memcpy(&out[i], q, 4); break;
                case 5: { double v; std::memcpy(&v, q, 8); out[i] = (float)v; break; }
                default: { uint16_t v; std::memcpy(&v, q, 2); uint32_t b = (uint32_t)v << 16; std::memcpy(&out[i], &b, 4); }
            }
        }
        return out;
    }

private:
    static float half_to_f32(uint16_t h) {
        const uint32_t sign = (uint32_t)(h >> 15) << 31, exp = (h >> 10) & 0x1F, man = h & 0x3FF;
        uint32_t bits;
        if (exp == 0) {
            if (man == 0) bits = sign;
            else {  // subnormal
                int e = -1;
                uint32_t m = man;
                do { ++e; m <<= 1; } while (!(m & 0x400));
                bits = sign | ((uint32_t)(127 - 15 - e) << 23) | ((m & 0x3FF) << 13);
            }
        } else if (exp == 31) bits = sign | 0x7F800000u | (man << 13);
        else bits = sign | ((exp + 112) << 23) | (man << 13);
        float f;
        std::memcpy(&f, &bits, 4);
        return f;
    }
    static bool known_dtype(uint32_t c) { return c == 0 || c == 1 || c == 8 || c == 12 || c == 14 || c == 16; }
    static size_t block_of(int q) { return q == DSQ_Q8_0 ? 32 : (q == DSQ_Q4K || q == DSQ_Q6K) ? 256 : 0; }

    size_t pos_ = 0;
    void need(size_t n) {
        if (pos_ + n > size_) throw std::runtime_error("EINVAL: snapshot malformed: truncated at byte " + std::to_string(pos_));
    }
    uint32_t u32() { need(4); uint32_t v; std::memcpy(&v, data_ + pos_, 4); pos_ += 4; return v; }
    uint64_t u64() { need(8); uint64_t v; std::memcpy(&v, data_ + pos_, 8); pos_ += 8; return v; }
    std::string str() {
        const uint32_t n = u32();
        need(n);
        std::string s(reinterpret_cast<const char*>(data_ + pos_), n);
        pos_ += n;
        return s;
    }

    void parse() {
        need(7);
        if (std::memcmp(data_, "DSQSNAP", 7) != 0) throw std::runtime_error("EINVAL: invalid snapshot magic in " + path_);
        pos_ = 7;
        const uint32_t version = u32();
        if (version != 1)
            throw std::runtime_error("EINVAL: unsupported snapshot version " + std::to_string(version) + ", expected 1");
        candle_version_ = str();
        model_id_ = str();
        backend_ = str();
        const uint32_t dq = u32();
        if (!known_dtype(dq)) throw std::runtime_error("EINVAL: unsupported tensor dtype code " + std::to_string(dq));
        default_qdtype_ = (int)dq;
        const uint32_t bs = u32();
        if (bs == 0) throw std::runtime_error("EINVAL: snapshot validation failed: block_size must be non-zero");
        const uint32_t count = u32();
        records_.reserve(count);
        for (uint32_t i = 0; i < count; ++i) {
            DsqRecord r;
            r.name = str();
            r.out_dim = u32();
            r.in_dim = u32();
            const uint32_t qd = u32();
            if (!known_dtype(qd)) throw std::runtime_error("EINVAL: unsupported tensor dtype code " + std::to_string(qd));
            r.q_dtype = (int)qd;
            r.q_offset = u64();
            r.q_len = u64();
            const uint64_t bo = u64(), bl = u64();
            const uint32_t bd = u32();
            if (bl != 0) {
                if (bd > 6) throw std::runtime_error("EINVAL: unsupported bias dtype code " + std::to_string(bd));
                r.has_bias = true;
                r.bias_offset = bo;
                r.bias_len = bl;
                r.bias_dtype = (int)bd;
            }
            records_.push_back(std::move(r));
        }
        const size_t meta = pos_;
        const size_t eb = block_of(default_qdtype_);
        if (!eb) throw std::runtime_error("EINVAL: snapshot validation failed: default dtype not quantised");
        if (bs != eb)
            throw std::runtime_error("EINVAL: snapshot validation failed: block size " + std::to_string(bs) +
                                     " mismatches expected " + std::to_string(eb));
        for (size_t i = 0; i < records_.size(); ++i) {
            const DsqRecord& r = records_[i];
            const std::string tn = "tensor `" + r.name + "` ";
            if (r.q_len == 0) throw std::runtime_error("EINVAL: " + tn + "has empty quantized payload");
            if (r.q_offset < meta) throw std::runtime_error("EINVAL: " + tn + "q_offset overlaps metadata");
            if (r.q_offset > size_ || r.q_len > size_ - r.q_offset)
                throw std::runtime_error("EINVAL: " + tn + "quantized slice exceeds file size");
            if (r.has_bias && (r.bias_offset > size_ || r.bias_len > size_ - r.bias_offset))
                throw std::runtime_error("EINVAL: " + tn + "bias slice exceeds file size");
            const size_t rb = block_of(r.q_dtype);
            if (rb) {
                if (r.in_dim % rb)
                    throw std::runtime_error("EINVAL: " + tn + "in_dim " + std::to_string(r.in_dim) +
                                             " not divisible by block_size " + std::to_string(rb));
            } else if (r.q_len != dsq_payload_bytes(r.q_dtype, r.out_dim, r.in_dim)) {
                throw std::runtime_error("EINVAL: " + tn + "has q_len " + std::to_string(r.q_len) +
                                         " but expected " + std::to_string(dsq_payload_bytes(r.q_dtype, r.out_dim, r.in_dim)));
            }
            if (!index_.emplace(r.name, i).second) throw std::runtime_error("EINVAL: duplicate tensor record `" + r.name + "`");
        }
    }

    std::string path_;
    int fd_ = -1;
    size_t size_ = 0;
    const uint8_t* data_ = nullptr;
    std::string candle_version_, model_id_, backend_;
    int default_qdtype_ = 0;
    std::vector<DsqRecord> records_;
    std::map<std::string, size_t> index_;
};

}  // namespace dsocr
