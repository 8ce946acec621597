// Host-side page preprocessing (a1-a3) and the one-time table resizes the vision
// tower needs.  Integer work is bit-exact with the reference:
//   resize_bicubic        vision/resample.rs:44-160 (Pillow 22-bit fixed point)
//   build_global_view     model/mod.rs:2295-2330
//   dynamic_preprocess    vision/preprocess.rs:67-138 (PreprocessParams::ocr1)
//   image_to_tensor       model/mod.rs:2332-2347
//   bicubic_resize_aa     vision/sam.rs:1000-1123 (pos-embed tables, f32)
//   rel_pos_resize        vision/sam.rs:1194-1232 (linear, f32)
#pragma once
#include <cmath>
#include <cstdint>
#include <set>
#include <utility>
#include <vector>

namespace dsocr {

struct ResampleCoeffs {
    std::vector<std::pair<int, int>> bounds;
    std::vector<int32_t> coeffs;
    int ksize = 0;
};

inline double bicubic_kernel_f64(double v) {
    const double A = -0.5;
    double x = std::fabs(v);
    if (x < 1.0) return ((A + 2.0) * x - (A + 3.0)) * x * x + 1.0;
    if (x < 2.0) return (((x - 5.0) * x + 8.0) * x - 4.0) * A;
    return 0.0;
}

inline long round_half_towards_zero(double v) { return v >= 0.0 ? (long)std::floor(v + 0.5) : (long)std::ceil(v + 0.5); }

inline ResampleCoeffs compute_resample_coeffs(int in_size, int out_size) {
    ResampleCoeffs rc;
    const double scale = (double)in_size / (double)out_size;
    const double filterscale = scale > 1.0 ? scale : 1.0;
    const double support = 2.0 * filterscale;
    rc.ksize = (int)std::ceil(support) * 2 + 1;
    rc.coeffs.assign((size_t)out_size * rc.ksize, 0);
    std::vector<double> row(rc.ksize);
    for (int o = 0; o < out_size; ++o) {
        const double center = (o + 0.5) * scale;
        long xmin = round_half_towards_zero(center - support);
        if (xmin < 0) xmin = 0;
        long xmax = round_half_towards_zero(center + support);
        if (xmax > in_size) xmax = in_size;
        if (xmin >= in_size) xmin = in_size > 0 ? in_size - 1 : 0;
        if (xmax <= xmin) xmax = xmin + 1;
        const int length = (int)(xmax - xmin);
        const double ss = 1.0 / filterscale;
        std::fill(row.begin(), row.end(), 0.0);
        double sum = 0.0;
        for (int i = 0; i < length && i < rc.ksize; ++i) {
            double w = bicubic_kernel_f64(((double)xmin + i - center + 0.5) * ss);
            row[i] = w;
            sum += w;
        }
        if (sum != 0.0)
            for (int i = 0; i < length && i < rc.ksize; ++i) row[i] /= sum;
        for (int i = 0; i < rc.ksize; ++i) {
            double v = row[i];
            rc.coeffs[(size_t)o * rc.ksize + i] = v < 0.0 ? (int32_t)(-0.5 + v * 4194304.0) : (int32_t)(0.5 + v * 4194304.0);
        }
        rc.bounds.push_back({(int)xmin, length});
    }
    return rc;
}

inline uint8_t clip8(int64_t v) {
    int64_t s = v >> 22;
    return (uint8_t)(s < 0 ? 0 : (s > 255 ? 255 : s));
}

// src HWC RGB8 (sw x sh) -> dst (dw x dh)
inline void resize_bicubic(const uint8_t* src, int sw, int sh, uint8_t* dst, int dw, int dh) {
    if (dw == 0 || dh == 0) return;
    ResampleCoeffs cx = compute_resample_coeffs(sw, dw), cy = compute_resample_coeffs(sh, dh);
    std::vector<uint8_t> hz((size_t)sh * dw * 3);
    const int64_t bias = (int64_t)1 << 21;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < sh; ++y) {
        const uint8_t* srow = src + (size_t)y * sw * 3;
        for (int x = 0; x < dw; ++x) {
            const int start = cx.bounds[x].first, len = cx.bounds[x].second;
            const int32_t* co = &cx.coeffs[(size_t)x * cx.ksize];
            int64_t a0 = bias, a1 = bias, a2 = bias;
            for (int i = 0; i < len; ++i) {
                const uint8_t* p = srow + (size_t)(start + i) * 3;
                a0 += (int64_t)p[0] * co[i];
                a1 += (int64_t)p[1] * co[i];
                a2 += (int64_t)p[2] * co[i];
            }
            uint8_t* d = &hz[((size_t)y * dw + x) * 3];
            d[0] = clip8(a0); d[1] = clip8(a1); d[2] = clip8(a2);
        }
    }
#pragma omp parallel for schedule(static)
    for (int y = 0; y < dh; ++y) {
        const int start = cy.bounds[y].first, len = cy.bounds[y].second;
        const int32_t* co = &cy.coeffs[(size_t)y * cy.ksize];
        for (int x = 0; x < dw; ++x) {
            int64_t a0 = bias, a1 = bias, a2 = bias;
            for (int i = 0; i < len; ++i) {
                const uint8_t* p = &hz[((size_t)(start + i) * dw + x) * 3];
                a0 += (int64_t)p[0] * co[i];
                a1 += (int64_t)p[1] * co[i];
                a2 += (int64_t)p[2] * co[i];
            }
            uint8_t* d = dst + ((size_t)y * dw + x) * 3;
            d[0] = clip8(a0); d[1] = clip8(a1); d[2] = clip8(a2);
        }
    }
}

// ---------------------------------------------------------------------------------------------------
// dots.ocr page resize (crates/infer-dots/src/vision/preprocess.rs:283-299): fast_image_resize 5.3.0
// (Cargo.lock) ResizeAlg::Convolution(FilterType::CatmullRom) on U8x3, restated from that crate's
// published algorithm (the crate is not in the repository: parity unpinned):
//   * per axis: scale = in / out, filter scale = max(scale, 1), radius = 2 * filter scale; output x
//     centres at (x + 0.5) * scale, taps floor(centre - radius) .. ceil(centre + radius) clamped to the
//     image, weight k((i - centre + 0.5) / filter scale) with the Catmull-Rom cubic (B = 0, C = 0.5),
//     normalised to sum 1;
//   * the weights become i16 at the largest precision p <= 14 whose doubled maximum still fits
//     (round half away from zero), the accumulator starts at 2^(p-1), the result is acc >> p clamped to
//     0..255;
//   * horizontal pass first into an 8-bit image, then the vertical pass.
// Against Pillow's bicubic (the same cubic at 22-bit precision, resize_bicubic above) the two differ
// only in rounding: tests/test_dots.py::test_fir_catmull_rom_vs_pillow states by how much.
inline double catmull_rom_fir(double x) {
    const double B = 0.0, C = 0.5;
    x = std::fabs(x);
    if (x < 1.0) return ((12.0 - 9.0 * B - 6.0 * C) * x * x * x + (-18.0 + 12.0 * B + 6.0 * C) * x * x + (6.0 - 2.0 * B)) / 6.0;
    if (x < 2.0)
        return ((-B - 6.0 * C) * x * x * x + (6.0 * B + 30.0 * C) * x * x + (-12.0 * B - 48.0 * C) * x + (8.0 * B + 24.0 * C)) /
               6.0;
    return 0.0;
}

struct FirCoeffs {
    std::vector<int> start, size;
    std::vector<std::vector<int16_t>> w;
    int precision = 0;
};

inline FirCoeffs fir_coeffs(int in_size, int out_size) {
    FirCoeffs fc;
    const double scale = (double)in_size / (double)out_size;
    const double fscale = std::max(scale, 1.0);
    const double radius = 2.0 * fscale;
    std::vector<std::vector<double>> wd((size_t)out_size);
    double max_w = 0.0;
    for (int x = 0; x < out_size; ++x) {
        const double centre = ((double)x + 0.5) * scale;
        const long x0 = std::max(0L, (long)std::floor(centre - radius));
        const long x1 = std::min((long)in_size, (long)std::ceil(centre + radius));
        double sum = 0.0;
        for (long i = x0; i < x1; ++i) {
            const double v = catmull_rom_fir(((double)i - centre + 0.5) / fscale);
            wd[x].push_back(v);
            sum += v;
        }
        if (sum != 0.0)
            for (double& v : wd[x]) v /= sum;
        for (double v : wd[x]) max_w = std::max(max_w, v);
        fc.start.push_back((int)x0);
        fc.size.push_back((int)(x1 - x0));
    }
    int precision = 0;
    for (int cur = 0; cur < 15; ++cur) {
        precision = cur;
        if (std::round(max_w * (double)(1 << (cur + 1))) >= (double)(1 << 15)) break;
    }
    fc.precision = precision;
    const double sc = (double)(1 << precision);
    fc.w.resize((size_t)out_size);
    for (int x = 0; x < out_size; ++x)
        for (double v : wd[x]) fc.w[x].push_back((int16_t)std::round(v * sc));  // std::round: half away from zero
    return fc;
}

inline uint8_t fir_clip(int32_t v, int precision) {
    const int32_t s = v >> precision;
    return (uint8_t)(s < 0 ? 0 : (s > 255 ? 255 : s));
}

// src HWC RGB8 (sw x sh) -> dst (dw x dh)
inline void resize_catmull_rom_fir(const uint8_t* src, int sw, int sh, uint8_t* dst, int dw, int dh) {
    if (dw <= 0 || dh <= 0) return;
    const FirCoeffs cx = fir_coeffs(sw, dw), cy = fir_coeffs(sh, dh);
    std::vector<uint8_t> hz((size_t)sh * dw * 3);
    if (dw == sw) {
        std::copy(src, src + (size_t)sh * sw * 3, hz.begin());
    } else {
        const int32_t init = 1 << (cx.precision - 1);
        for (int y = 0; y < sh; ++y)
            for (int x = 0; x < dw; ++x) {
                int32_t acc[3] = {init, init, init};
                const uint8_t* row = src + ((size_t)y * sw + cx.start[x]) * 3;
                for (int i = 0; i < cx.size[x]; ++i)
                    for (int c = 0; c < 3; ++c) acc[c] += (int32_t)row[i * 3 + c] * (int32_t)cx.w[x][i];
                for (int c = 0; c < 3; ++c) hz[((size_t)y * dw + x) * 3 + c] = fir_clip(acc[c], cx.precision);
            }
    }
    if (dh == sh) {
        std::copy(hz.begin(), hz.end(), dst);
        return;
    }
    const int32_t init = 1 << (cy.precision - 1);
    for (int y = 0; y < dh; ++y)
        for (int x = 0; x < dw; ++x) {
            int32_t acc[3] = {init, init, init};
            for (int i = 0; i < cy.size[y]; ++i) {
                const uint8_t* px = hz.data() + ((size_t)(cy.start[y] + i) * dw + x) * 3;
                for (int c = 0; c < 3; ++c) acc[c] += (int32_t)px[c] * (int32_t)cy.w[y][i];
            }
            for (int c = 0; c < 3; ++c) dst[((size_t)y * dw + x) * 3 + c] = fir_clip(acc[c], cy.precision);
        }
}

inline double round_ties_to_even(double v) {
    double r = std::round(v);  // half away from zero, like Rust f64::round
    if (std::fabs(v - r) != 0.5) return r;
    double t = std::trunc(v);
    return ((long)t % 2 == 0) ? t : t + (v > 0 ? 1.0 : -1.0);
}

// model/mod.rs:2308-2330: size and placement of the resized page on the base x base canvas
inline void global_view_geometry(int w, int h, int base, int* nw, int* nh, int* xo, int* yo) {
    double scale = std::min((double)base / w, (double)base / h);
    *nw = (int)std::min(std::max(round_ties_to_even(w * scale), 1.0), (double)base);
    *nh = (int)std::min(std::max(round_ties_to_even(h * scale), 1.0), (double)base);
    *xo = (int)round_ties_to_even((base - *nw) * 0.5);
    *yo = (int)round_ties_to_even((base - *nh) * 0.5);
}

inline std::vector<uint8_t> build_global_view(const uint8_t* rgb, int w, int h, int base) {
    const uint8_t mean = (uint8_t)(0.5 * 255.0);
    std::vector<uint8_t> canvas((size_t)base * base * 3, mean);
    if (w == 0 || h == 0) return canvas;
    int nw, nh, xo, yo;
    global_view_geometry(w, h, base, &nw, &nh, &xo, &yo);
    std::vector<uint8_t> rs((size_t)nw * nh * 3);
    resize_bicubic(rgb, w, h, rs.data(), nw, nh);
    for (int y = 0; y < nh; ++y) {
        int cyy = y + yo;
        if (cyy < 0 || cyy >= base) continue;
        for (int x = 0; x < nw; ++x) {
            int cxx = x + xo;
            if (cxx < 0 || cxx >= base) continue;
            for (int c = 0; c < 3; ++c) canvas[((size_t)cyy * base + cxx) * 3 + c] = rs[((size_t)y * nw + x) * 3 + c];
        }
    }
    return canvas;
}

// vision/preprocess.rs:67-138: the tile grid (closest aspect ratio, larger grid on ties when the
// page area exceeds half of it); false when the page needs no tiles
inline bool choose_tile_grid(int w, int h, int tile, int min_num, int max_num, int* grid_w, int* grid_h) {
    if (w <= tile && h <= tile) { *grid_w = 1; *grid_h = 1; return false; }
    const double aspect = (double)w / (double)h;
    std::set<std::pair<int, int>> ratios;
    for (int n = min_num; n <= max_num; ++n)
        for (int i = 1; i <= n; ++i)
            for (int j = 1; j <= n; ++j)
                if (i * j <= max_num && i * j >= min_num) ratios.insert({i, j});
    std::pair<int, int> best{1, 1};
    double best_diff = 1.79769313486231570e+308;
    const double area = (double)((long)w * h);
    for (auto& r : ratios) {
        double diff = std::fabs(aspect - (double)r.first / (double)r.second);
        if (diff < best_diff) { best_diff = diff; best = r; }
        else if (std::fabs(diff - best_diff) < 2.220446049250313e-16 &&
                 area > 0.5 * (double)((long)tile * tile * r.first * r.second))
            best = r;
    }
    *grid_w = best.first;
    *grid_h = best.second;
    return true;
}

// vision/preprocess.rs:67-138 -> tiles (row-major) and grid (w, h)
inline std::vector<std::vector<uint8_t>> dynamic_preprocess(const uint8_t* rgb, int w, int h, int tile, int min_num,
                                                            int max_num, int* grid_w, int* grid_h) {
    std::vector<std::vector<uint8_t>> tiles;
    if (!choose_tile_grid(w, h, tile, min_num, max_num, grid_w, grid_h)) return tiles;
    const std::pair<int, int> best{*grid_w, *grid_h};
    const int tw = tile * best.first, th = tile * best.second;
    std::vector<uint8_t> rs((size_t)tw * th * 3);
    resize_bicubic(rgb, w, h, rs.data(), tw, th);
    for (int i = 0; i < best.first * best.second; ++i) {
        int x0 = (i % best.first) * tile, y0 = (i / best.first) * tile;
        std::vector<uint8_t> t((size_t)tile * tile * 3);
        for (int y = 0; y < tile; ++y)
            std::copy(&rs[((size_t)(y0 + y) * tw + x0) * 3], &rs[((size_t)(y0 + y) * tw + x0 + tile) * 3], &t[(size_t)y * tile * 3]);
        tiles.push_back(std::move(t));
    }
    *grid_w = best.first;
    *grid_h = best.second;
    return tiles;
}

// model/mod.rs:2332-2347: CHW f32, (v/255 - 0.5)/0.5
inline void image_to_chw(const uint8_t* rgb, int w, int h, float* out) {
    for (int c = 0; c < 3; ++c)
        for (int y = 0; y < h; ++y)
            for (int x = 0; x < w; ++x) {
                float v = (float)rgb[((size_t)y * w + x) * 3 + c] / 255.0f;
                out[((size_t)c * h + y) * w + x] = (v - 0.5f) / 0.5f;
            }
}

// build_image_placeholders (model/mod.rs:2605-2689, Ocr1): number of <image> slots.
inline size_t image_placeholder_count(int base, int image_size, bool crop_mode, int cw, int ch) {
    const int P = 16, D = 4;
    size_t n = 0;
    if (crop_mode) {
        int ng = (int)std::ceil((float)(base / P) / (float)D);
        int nl = (int)std::ceil((float)(image_size / P) / (float)D);
        if (cw > 1 || ch > 1) n += (size_t)(nl * ch) * (nl * cw + 1);
        n += (size_t)ng * (ng + 1) + 1;
    } else {
        int nq = (int)std::ceil((float)(image_size / P) / (float)D);
        n += (size_t)nq * (nq + 1) + 1;
    }
    return n;
}

// ---------------------------------------------------------------- f32 table resizes
inline float bicubic_filter_pillow(float x) {
    const float a = -0.5f;
    x = std::fabs(x);
    if (x < 1.0f) return ((a + 2.0f) * x - (a + 3.0f)) * x * x + 1.0f;
    if (x < 2.0f) return (((x - 5.0f) * x + 8.0f) * x - 4.0f) * a;
    return 0.0f;
}
inline void axis_weights_aa(int in_len, int out_len, float scale, std::vector<std::vector<float>>& w,
                            std::vector<std::vector<int>>& idx) {
    const float support = scale >= 1.0f ? 2.0f * scale : 2.0f;
    const float invscale = scale >= 1.0f ? 1.0f / scale : 1.0f;
    w.assign(out_len, {});
    idx.assign(out_len, {});
    for (int o = 0; o < out_len; ++o) {
        const float center = scale * ((float)o + 0.5f);
        long xmin = (long)std::floor(center - support + 0.5f);
        if (xmin < 0) xmin = 0;
        long xmax = (long)std::floor(center + support + 0.5f);
        if (xmax > in_len) xmax = in_len;
        long xs = xmax > xmin ? xmax - xmin : 0;
        const float xmc = (float)xmin - center;
        float total = 0.f;
        for (long j = 0; j < xs; ++j) {
            float arg = ((float)j + xmc + 0.5f) * invscale;
            float ww = bicubic_filter_pillow(arg);
            w[o].push_back(ww);
            idx[o].push_back((int)(xmin + j));
            total += ww;
        }
        if (total != 0.f)
            for (auto& ww : w[o]) ww /= total;
    }
}
// in [C][in_h][in_w] -> out [C][out_h][out_w] (vertical pass, then horizontal; sam.rs:1084-1116)
inline std::vector<float> bicubic_resize_aa(const std::vector<float>& in, int C, int in_h, int in_w, int out_h,
                                            int out_w) {
    if (in_h == out_h && in_w == out_w) return in;
    std::vector<std::vector<float>> wy, wx;
    std::vector<std::vector<int>> iy, ix;
    axis_weights_aa(in_h, out_h, (float)in_h / (float)out_h, wy, iy);
    axis_weights_aa(in_w, out_w, (float)in_w / (float)out_w, wx, ix);
    std::vector<float> tmp((size_t)C * out_h * in_w), out((size_t)C * out_h * out_w);
#pragma omp parallel for schedule(static)
    for (int c = 0; c < C; ++c) {
        std::vector<float> acc(in_w);
        for (int oh = 0; oh < out_h; ++oh) {
            std::fill(acc.begin(), acc.end(), 0.f);
            for (size_t k = 0; k < iy[oh].size(); ++k) {
                const float wt = wy[oh][k];
                const float* r = &in[((size_t)c * in_h + iy[oh][k]) * in_w];
                for (int x = 0; x < in_w; ++x) acc[x] += r[x] * wt;
            }
            std::copy(acc.begin(), acc.end(), &tmp[((size_t)c * out_h + oh) * in_w]);
        }
        for (int oh = 0; oh < out_h; ++oh)
            for (int ow = 0; ow < out_w; ++ow) {
                float v = 0.f;
                for (size_t k = 0; k < ix[ow].size(); ++k) v += tmp[((size_t)c * out_h + oh) * in_w + ix[ow][k]] * wx[ow][k];
                out[((size_t)c * out_h + oh) * out_w + ow] = v;
            }
    }
    return out;
}
// get_rel_pos_vec resize part (sam.rs:1194-1232): [orig][hd] -> [2*size-1][hd]
inline std::vector<float> rel_pos_resize(const std::vector<float>& rel, int orig, int hd, int size) {
    const int max_rel = 2 * size - 1;
    if (orig == max_rel) return rel;
    std::vector<float> out((size_t)max_rel * hd);
    const float scale = (float)orig / (float)max_rel;
    for (int i = 0; i < max_rel; ++i) {
        float src = scale * ((float)i + 0.5f) - 0.5f;
        if (src < 0.f) src = 0.f;
        const float mx = (float)(orig - 1);
        if (src > mx) src = mx;
        const float lf = std::floor(src);
        const int left = (int)lf;
        const int right = std::min(left + 1, orig - 1);
        float w = src - lf;
        w = w < 0.f ? 0.f : (w > 1.f ? 1.f : w);
        for (int d = 0; d < hd; ++d) out[(size_t)i * hd + d] = rel[(size_t)left * hd + d] * (1.0f - w) + rel[(size_t)right * hd + d] * w;
    }
    return out;
}

}  // namespace dsocr
