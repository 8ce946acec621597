// Host helpers: half-precision conversions, safetensors mmap reader and the
// deterministic synthetic-weight generator (same published recipe as the
// oracle's synth.c; tests/test_host_cpu.py::test_synth_recipe_product_equals_oracle checks equality).
#pragma once
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "json.hpp"

namespace dsocr {

inline float bf16_to_f32(uint16_t h) {
    uint32_t u = (uint32_t)h << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

inline uint16_t f32_to_bf16_rne(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)((u >> 16) | ((u & 0xffff) ? 0x40 : 0));
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

// IEEE binary16, round-to-nearest-even (matches `half` crate / numpy astype(float16)).
inline uint16_t f32_to_f16_rne(float f) {
    uint32_t x;
    std::memcpy(&x, &f, 4);
    uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t mant = x & 0x007fffffu;
    int32_t exp = (int32_t)((x >> 23) & 0xff);
    if (exp == 0xff) return (uint16_t)(sign | 0x7c00u | (mant ? 0x200u : 0u));
    int32_t e = exp - 127 + 15;
    if (e >= 31) return (uint16_t)(sign | 0x7c00u);
    if (e <= 0) {
        if (e < -10) return (uint16_t)sign;
        mant |= 0x00800000u;
        uint32_t shift = (uint32_t)(14 - e);
        uint32_t half_m = mant >> shift;
        uint32_t rem = mant & ((1u << shift) - 1u);
        uint32_t halfway = 1u << (shift - 1);
        if (rem > halfway || (rem == halfway && (half_m & 1u))) half_m++;
        return (uint16_t)(sign | half_m);
    }
    uint32_t half_m = mant >> 13;
    uint32_t rem = mant & 0x1fffu;
    uint16_t out = (uint16_t)(sign | ((uint32_t)e << 10) | half_m);
    if (rem > 0x1000u || (rem == 0x1000u && (half_m & 1u))) out++;
    return out;
}

inline float f16_to_f32(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t exp = (h >> 10) & 0x1f;
    uint32_t mant = h & 0x3ffu;
    uint32_t u;
    if (exp == 0) {
        if (mant == 0) {
            u = sign;
        } else {
            int e = -1;
            do { e++; mant <<= 1; } while (!(mant & 0x400u));
            mant &= 0x3ffu;
            u = sign | ((uint32_t)(127 - 15 - e) << 23) | (mant << 13);
        }
    } else if (exp == 0x1f) {
        u = sign | 0x7f800000u | (mant << 13);
    } else {
        u = sign | ((exp - 15 + 127) << 23) | (mant << 13);
    }
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

// --------------------------------------------------------------------------- synthetic weights
inline uint64_t fnv1a64(const std::string& s) {
    uint64_t h = 1469598103934665603ULL;
    for (unsigned char c : s) { h ^= c; h *= 1099511628211ULL; }
    return h;
}
inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
// Init rule: norm weights ~ 1 + N(0, 0.05), everything else N(0, 0.02).
inline void synth_init_rule(const std::string& name, double* mean, double* stdv) {
    auto ends = [&](const char* s) { size_t n = strlen(s); return name.size() >= n && name.compare(name.size() - n, n, s) == 0; };
    bool norm_w = ends(".weight") && (name.find("norm") != std::string::npos || name.find(".neck.1.") != std::string::npos ||
                                      name.find(".neck.3.") != std::string::npos || name.find(".ln_q.") != std::string::npos);
    *mean = norm_w ? 1.0 : 0.0;
    *stdv = norm_w ? 0.05 : 0.02;
}
inline void synth_bf16(const std::string& name, uint64_t seed, uint64_t n, uint16_t* out) {
    double mean, stdv;
    synth_init_rule(name, &mean, &stdv);
    const uint64_t key = fnv1a64(name) ^ (seed * 0x9E3779B97F4A7C15ULL);
    const float scale = (float)(stdv / 147.80);
    const float fmean = (float)mean;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        uint64_t z = mix64(key + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ULL);
        int c = (int)(z & 0xff) + (int)((z >> 8) & 0xff) + (int)((z >> 16) & 0xff) + (int)((z >> 24) & 0xff) - 510;
        float v = (float)c * scale;
        v = v + fmean;
        out[i] = f32_to_bf16_rne(v);
    }
}
// Which optional tensors a synthetic checkpoint carries (see oracle/weights.py synthetic_has).
inline bool synth_has(const std::string& name) {
    auto ends = [&](const char* s) { size_t n = strlen(s); return name.size() >= n && name.compare(name.size() - n, n, s) == 0; };
    if (name.rfind("model.layers.", 0) == 0 && ends(".bias")) return false;
    if (name.find("e_score_correction_bias") != std::string::npos) return false;
    if (name.find("vision_model.embeddings.patch_embedding") != std::string::npos) return false;
    return true;
}

// --------------------------------------------------------------------------- safetensors
struct StTensor {
    std::string dtype;  // "BF16", "F16", "F32"
    std::vector<int64_t> shape;
    const uint8_t* data = nullptr;
    size_t nbytes = 0;
    int64_t numel() const { int64_t n = 1; for (auto s : shape) n *= s; return n; }
};

class SafeTensors {
  public:
    explicit SafeTensors(const std::string& path) {
        fd_ = ::open(path.c_str(), O_RDONLY);
        if (fd_ < 0) throw std::runtime_error("ENOENT: cannot open weights " + path);
        struct stat st;
        fstat(fd_, &st);
        size_ = (size_t)st.st_size;
        map_ = (uint8_t*)mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd_, 0);
        if (map_ == MAP_FAILED) throw std::runtime_error("mmap failed for " + path);
        if (size_ < 8) throw std::runtime_error("safetensors file too small");
        uint64_t hlen;
        std::memcpy(&hlen, map_, 8);
        if (8 + hlen > size_) throw std::runtime_error("safetensors header overflows file");
        Json h = Json::parse((const char*)map_ + 8, hlen);
        const uint8_t* base = map_ + 8 + hlen;
        for (auto& kv : h.obj) {
            if (kv.first == "__metadata__") continue;
            StTensor t;
            t.dtype = kv.second["dtype"].as_string();
            for (auto& d : kv.second["shape"].arr) t.shape.push_back(d.as_int());
            size_t s = (size_t)kv.second["data_offsets"][0].as_int();
            size_t e = (size_t)kv.second["data_offsets"][1].as_int();
            if (base + e > map_ + size_) throw std::runtime_error("tensor data out of range: " + kv.first);
            t.data = base + s;
            t.nbytes = e - s;
            tensors_[kv.first] = t;
        }
    }
    ~SafeTensors() {
        if (map_ && map_ != MAP_FAILED) munmap(map_, size_);
        if (fd_ >= 0) ::close(fd_);
    }
    bool has(const std::string& n) const { return tensors_.count(n) != 0; }
    const StTensor& get(const std::string& n) const {
        auto it = tensors_.find(n);
        if (it == tensors_.end()) throw std::runtime_error("ENOENT: missing tensor `" + n + "`");
        return it->second;
    }

  private:
    int fd_ = -1;
    size_t size_ = 0;
    uint8_t* map_ = nullptr;
    std::map<std::string, StTensor> tensors_;
};

}  // namespace dsocr
