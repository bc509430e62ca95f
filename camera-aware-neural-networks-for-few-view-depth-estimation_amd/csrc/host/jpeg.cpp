// Sequential-Huffman JPEG decoder for the data path.
//
// The reference reads SUN RGB-D's RGB frames with cv::imread(path, cv::IMREAD_COLOR)
// (src/data/sunrgbd_loader.cpp:86,222), i.e. libjpeg-turbo's default decompression.  This decoder
// restates that pipeline so the decoded bytes are identical:
//   * entropy decoding of baseline / extended-sequential Huffman scans (ITU-T T.81 Annex F: DHT,
//     DQT with 8- or 16-bit tables, DRI restart intervals, interleaved and single-component scans),
//     coefficients truncated to 16 bits as libjpeg's JCOEF;
//   * the ISLOW integer inverse DCT (libjpeg jidctint.c algorithm: 13-bit constants, 2 extra bits in
//     the column pass, outputs through the wrap-around range-limit table);
//   * "fancy" chroma upsampling (jdsample.c: triangle filters h2v1 / h2v2 / h1v2 with their rounding
//     biases, box replication where libjpeg-turbo uses it), edge rows and columns replicated as the
//     main controller's context rows are;
//   * YCbCr -> RGB through the fixed-point tables of jdcolor.c (16 fraction bits);
//   * JFIF / Adobe APP14 / component-id colour-space inference (jdapimin.c default_decompress_parms).
//   * progressive Huffman scans (T.81 Annex G; libjpeg jdphuff.c): DC first / refinement scans
//     (interleaved or not), AC first scans with end-of-band runs and AC refinement scans with their
//     correction bits, coefficients kept for the whole image until the last scan; the same IDCT and
//     upsampling then apply.
// Not supported (clear error): lossless processes, arithmetic coding, 12-bit samples, CMYK / YCCK
// (SUN RGB-D's frames are baseline 8-bit YCbCr), and progressive files whose scans leave any of the
// first nine AC coefficients short of their last bit — libjpeg-turbo then applies its block
// smoothing (jdcoefct.c smoothing_ok), which this decoder does not restate; a complete progression
// (every standard encoder's script) refines every coefficient to bit 0.  The EXIF orientation tag is
// applied as cv::imread(IMREAD_COLOR) applies it.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "jpeg.hpp"

namespace cad {
namespace jpeg {

namespace {

struct JpegError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// zig-zag index -> natural (row-major) index, with 16 guard entries for corrupt run lengths
// (libjpeg's jpeg_natural_order)
constexpr int kNatural[80] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33,
                              40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36,
                              29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54,
                              47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

struct Huffman {
    bool defined = false;
    // code-length tables (T.81 F.2.2.3): maxcode[l] (-1: none), valoff[l]
    int32_t maxcode[18];
    int32_t valoff[18];
    uint8_t vals[256];
    // 9-bit lookahead: (length << 8) | value, 0 = longer code
    uint16_t look[512];

    // is_dc: a DC table's symbols are coefficient sizes, at most 15 (jdhuff.c jpeg_make_d_derived_tbl
    // rejects larger ones; a baseline decoder needs <= 11, checked where the symbol is used)
    void build(const uint8_t bits[17], const uint8_t* v, int nv, bool is_dc) {
        std::memcpy(vals, v, (size_t)nv);
        if (is_dc)
            for (int i = 0; i < nv; ++i)
                if (vals[i] > 15) throw JpegError("bad Huffman table (DC symbol > 15)");
        int code = 0, k = 0;
        std::memset(look, 0, sizeof look);
        for (int l = 1; l <= 16; ++l) {
            valoff[l] = k - code;
            // an over-full length is rejected before any lookahead entry is written: the codes of
            // length l must fit in l bits and none may be all ones (jdhuff.c jpeg_make_d_derived_tbl,
            // code >= 1 << si -> JERR_BAD_HUFF_TABLE)
            if (bits[l] && code + (int)bits[l] >= (1 << l)) throw JpegError("bad Huffman table");
            if (bits[l]) {
                for (int i = 0; i < bits[l]; ++i, ++code, ++k) {
                    if (l <= 9) {
                        const int base = code << (9 - l);
                        for (int j = 0; j < (1 << (9 - l)); ++j) look[base + j] = (uint16_t)(l << 8 | vals[k]);
                    }
                }
                maxcode[l] = code - 1;
            } else {
                maxcode[l] = -1;
            }
            code <<= 1;
        }
        maxcode[17] = 0x7FFFFFFF;   // sentinel
        defined = true;
    }
};

// Bit reader over entropy-coded data: 0xFF00 stuffing removed; at a marker it feeds zero bits (as
// libjpeg does after its "premature end of data" warning) without consuming the marker.
struct Bits {
    const uint8_t* p;
    const uint8_t* end;
    uint64_t acc = 0;
    int n = 0;
    bool at_marker = false;

    void fill() {
        while (n <= 56) {
            uint32_t b = 0;
            if (!at_marker && p < end) {
                b = *p;
                if (b == 0xFF) {
                    const uint32_t nb = p + 1 < end ? p[1] : 0xD9;
                    if (nb == 0x00) {
                        p += 2;
                    } else {
                        at_marker = true;
                        b = 0;
                    }
                } else {
                    ++p;
                }
            }
            acc |= (uint64_t)b << (56 - n);
            n += 8;
        }
    }
    int get(int k) {   // k <= 16
        if (k == 0) return 0;
        if (n < k) fill();
        const int v = (int)(acc >> (64 - k));
        acc <<= k;
        n -= k;
        return v;
    }
    int decode(const Huffman& h) {
        if (n < 16) fill();
        const int peek = (int)(acc >> (64 - 9));
        const uint16_t e = h.look[peek];
        if (e) {
            const int l = e >> 8;
            acc <<= l;
            n -= l;
            return e & 0xFF;
        }
        int code = (int)(acc >> (64 - 10));
        int l = 10;
        while (l <= 16 && code > h.maxcode[l]) {
            code = (int)(acc >> (64 - ++l));
        }
        if (l > 16) {   // corrupt data: libjpeg returns 0 and warns
            acc <<= 16;
            n -= 16;
            return 0;
        }
        acc <<= l;
        n -= l;
        return h.vals[(code + h.valoff[l]) & 0xFF];
    }
    void reset() {   // discard the rest of the byte-aligned segment (restart)
        acc = 0;
        n = 0;
    }
};

inline int extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

struct Component {
    int id = 0, h = 1, v = 1, tq = 0;
    int td = 0, ta = 0;             // Huffman table selectors of the current scan
    int bw = 0, bh = 0;             // blocks per row / column (padded to whole MCUs)
    int dw = 0, dh = 0;             // downsampled width / height (samples)
    std::vector<int16_t> coef;      // bw * bh * 64, natural order
    std::vector<uint8_t> plane;     // (8 bw) x (8 bh) samples
    int pred = 0;
    int coef_bits[64];              // progressive: the point transform Al of the last scan of each
                                    // coefficient (-1: not yet coded), libjpeg's coef_bits
};

// ------------------------------------------------------------------------------------------------
// progressive scans (jdphuff.c decode_mcu_DC_first / _DC_refine / _AC_first / _AC_refine); blk is
// one block's 64 coefficients in natural order, as JCOEF (16-bit) values
// ------------------------------------------------------------------------------------------------
void dc_first(Bits& bits, const Huffman& h, Component& c, int al, int16_t* blk) {
    const int t = bits.decode(h);
    if (t > 11) throw JpegError("bad DC coefficient");
    const int diff = t ? extend(bits.get(t), t) : 0;
    c.pred += diff;
    blk[0] = (int16_t)((uint32_t)c.pred << al);
}
void dc_refine(Bits& bits, int al, int16_t* blk) {
    if (bits.get(1)) blk[0] = (int16_t)(blk[0] | (1 << al));
}
void ac_first(Bits& bits, const Huffman& h, int ss, int se, int al, int& eobrun, int16_t* blk) {
    if (eobrun > 0) {   // a band of zeros
        --eobrun;
        return;
    }
    for (int k = ss; k <= se; ++k) {
        const int rs = bits.decode(h);
        const int r = rs >> 4, s = rs & 15;
        if (s) {
            k += r;
            blk[kNatural[k]] = (int16_t)((uint32_t)extend(bits.get(s), s) << al);
        } else if (r == 15) {   // ZRL: 16 zeros
            k += 15;
        } else {                // EOBr: 2^r + r appended bits blocks end here
            eobrun = 1 << r;
            if (r) eobrun += bits.get(r);
            --eobrun;
            break;
        }
    }
}
void ac_refine(Bits& bits, const Huffman& h, int ss, int se, int al, int& eobrun, int16_t* blk) {
    const int p1 = 1 << al, m1 = -(1 << al);
    // a correction bit for an already-nonzero coefficient: 1 = its magnitude grows by p1
    auto correct = [&](int16_t& v) {
        if (bits.get(1) && (v & p1) == 0) v = (int16_t)(v + (v >= 0 ? p1 : m1));
    };
    int k = ss;
    if (eobrun == 0) {
        for (; k <= se; ++k) {
            const int rs = bits.decode(h);
            int r = rs >> 4, s = rs & 15;
            if (s) {   // a newly nonzero coefficient of magnitude p1 (s should be 1)
                s = bits.get(1) ? p1 : m1;
            } else if (r != 15) {   // EOBr: the rest of this block is handled by the EOB logic below
                eobrun = 1 << r;
                if (r) eobrun += bits.get(r);
                break;
            }
            // advance over already-nonzero coefficients (correction bits) and r still-zero ones
            do {
                int16_t& v = blk[kNatural[k]];
                if (v != 0) {
                    correct(v);
                } else if (--r < 0) {
                    break;   // the target zero coefficient
                }
                ++k;
            } while (k <= se);
            if (s) blk[kNatural[k]] = (int16_t)s;
        }
    }
    if (eobrun > 0) {   // the remaining positions of a block inside an EOB run: correction bits only
        for (; k <= se; ++k) {
            int16_t& v = blk[kNatural[k]];
            if (v != 0) correct(v);
        }
        --eobrun;
    }
}

// ------------------------------------------------------------------------------------------------
// ISLOW inverse DCT (jidctint.c): CONST_BITS 13, PASS1_BITS 2; samples through the post-IDCT
// range-limit table (jdmaster.c prepare_range_limit_table: x & 1023 -> clamp(x + 128) with wrap)
// ------------------------------------------------------------------------------------------------
struct RangeLimit {
    uint8_t t[1024];
    RangeLimit() {
        for (int x = 0; x < 1024; ++x) {
            int v;
            if (x < 128) v = x + 128;
            else if (x < 512) v = 255;
            else if (x < 896) v = 0;
            else v = x - 896;
            t[x] = (uint8_t)v;
        }
    }
};
const RangeLimit kRange;

constexpr int64_t F0_298 = 2446, F0_390 = 3196, F0_541 = 4433, F0_765 = 6270, F0_899 = 7373, F1_175 = 9633,
                  F1_501 = 12299, F1_847 = 15137, F1_961 = 16069, F2_053 = 16819, F2_562 = 20995,
                  F3_072 = 25172;
constexpr int CB = 13, P1 = 2;
inline int64_t descale(int64_t x, int n) { return (x + ((int64_t)1 << (n - 1))) >> n; }

// quantiser multipliers are libjpeg's ISLOW_MULT_TYPE (short): a 16-bit table entry >= 32768 wraps
void idct_islow(const int16_t* in, const int16_t* q, uint8_t* out, int ostride) {
    int ws[64];
    for (int c = 0; c < 8; ++c) {
        const int16_t* ip = in + c;
        const int16_t* qp = q + c;
        int* wp = ws + c;
        if (!ip[8] && !ip[16] && !ip[24] && !ip[32] && !ip[40] && !ip[48] && !ip[56]) {
            const int dc = (int)((int)ip[0] * (int)qp[0]) * (1 << P1);
            for (int r = 0; r < 8; ++r) wp[8 * r] = dc;
            continue;
        }
        int64_t z2 = (int)ip[16] * (int)qp[16], z3 = (int)ip[48] * (int)qp[48];
        int64_t z1 = (z2 + z3) * F0_541;
        int64_t tmp2 = z1 + z3 * -F1_847;
        int64_t tmp3 = z1 + z2 * F0_765;
        z2 = (int)ip[0] * (int)qp[0];
        z3 = (int)ip[32] * (int)qp[32];
        int64_t tmp0 = (z2 + z3) * (1 << CB);
        int64_t tmp1 = (z2 - z3) * (1 << CB);
        const int64_t t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
        tmp0 = (int)ip[56] * (int)qp[56];
        tmp1 = (int)ip[40] * (int)qp[40];
        tmp2 = (int)ip[24] * (int)qp[24];
        tmp3 = (int)ip[8] * (int)qp[8];
        z1 = tmp0 + tmp3;
        z2 = tmp1 + tmp2;
        z3 = tmp0 + tmp2;
        int64_t z4 = tmp1 + tmp3;
        const int64_t z5 = (z3 + z4) * F1_175;
        tmp0 *= F0_298;
        tmp1 *= F2_053;
        tmp2 *= F3_072;
        tmp3 *= F1_501;
        z1 *= -F0_899;
        z2 *= -F2_562;
        z3 *= -F1_961;
        z4 *= -F0_390;
        z3 += z5;
        z4 += z5;
        tmp0 += z1 + z3;
        tmp1 += z2 + z4;
        tmp2 += z2 + z3;
        tmp3 += z1 + z4;
        wp[0] = (int)descale(t10 + tmp3, CB - P1);
        wp[56] = (int)descale(t10 - tmp3, CB - P1);
        wp[8] = (int)descale(t11 + tmp2, CB - P1);
        wp[48] = (int)descale(t11 - tmp2, CB - P1);
        wp[16] = (int)descale(t12 + tmp1, CB - P1);
        wp[40] = (int)descale(t12 - tmp1, CB - P1);
        wp[24] = (int)descale(t13 + tmp0, CB - P1);
        wp[32] = (int)descale(t13 - tmp0, CB - P1);
    }
    for (int r = 0; r < 8; ++r) {
        const int* wp = ws + 8 * r;
        uint8_t* op = out + r * ostride;
        if (!wp[1] && !wp[2] && !wp[3] && !wp[4] && !wp[5] && !wp[6] && !wp[7]) {
            const uint8_t v = kRange.t[(int)descale(wp[0], P1 + 3) & 1023];
            for (int c = 0; c < 8; ++c) op[c] = v;
            continue;
        }
        int64_t z2 = wp[2], z3 = wp[6];
        int64_t z1 = (z2 + z3) * F0_541;
        int64_t tmp2 = z1 + z3 * -F1_847;
        int64_t tmp3 = z1 + z2 * F0_765;
        int64_t tmp0 = ((int64_t)wp[0] + wp[4]) * (1 << CB);
        int64_t tmp1 = ((int64_t)wp[0] - wp[4]) * (1 << CB);
        const int64_t t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
        tmp0 = wp[7];
        tmp1 = wp[5];
        tmp2 = wp[3];
        tmp3 = wp[1];
        z1 = tmp0 + tmp3;
        z2 = tmp1 + tmp2;
        z3 = tmp0 + tmp2;
        int64_t z4 = tmp1 + tmp3;
        const int64_t z5 = (z3 + z4) * F1_175;
        tmp0 *= F0_298;
        tmp1 *= F2_053;
        tmp2 *= F3_072;
        tmp3 *= F1_501;
        z1 *= -F0_899;
        z2 *= -F2_562;
        z3 *= -F1_961;
        z4 *= -F0_390;
        z3 += z5;
        z4 += z5;
        tmp0 += z1 + z3;
        tmp1 += z2 + z4;
        tmp2 += z2 + z3;
        tmp3 += z1 + z4;
        constexpr int S = CB + P1 + 3;
        op[0] = kRange.t[(int)descale(t10 + tmp3, S) & 1023];
        op[7] = kRange.t[(int)descale(t10 - tmp3, S) & 1023];
        op[1] = kRange.t[(int)descale(t11 + tmp2, S) & 1023];
        op[6] = kRange.t[(int)descale(t11 - tmp2, S) & 1023];
        op[2] = kRange.t[(int)descale(t12 + tmp1, S) & 1023];
        op[5] = kRange.t[(int)descale(t12 - tmp1, S) & 1023];
        op[3] = kRange.t[(int)descale(t13 + tmp0, S) & 1023];
        op[4] = kRange.t[(int)descale(t13 - tmp0, S) & 1023];
    }
}

// ------------------------------------------------------------------------------------------------
// upsampling (jdsample.c) of one component plane (dw x dh real samples, row stride `ls`) to
// (dw * hx) x (dh * vx); rows above the first / below the last are the edge rows (context rows)
// ------------------------------------------------------------------------------------------------
std::vector<uint8_t> upsample(const Component& cp, int hx, int vx, bool fancy) {
    const int dw = cp.dw, dh = cp.dh, ls = cp.bw * 8;
    const int ow = dw * hx, oh = dh * vx;
    std::vector<uint8_t> o((size_t)ow * oh);
    auto row = [&](int r) { return cp.plane.data() + (size_t)(r < 0 ? 0 : r >= dh ? dh - 1 : r) * ls; };
    if (hx == 1 && vx == 1) {
        for (int r = 0; r < dh; ++r) std::memcpy(&o[(size_t)r * ow], row(r), (size_t)dw);
    } else if (hx == 2 && vx == 1) {
        for (int r = 0; r < dh; ++r) {
            const uint8_t* in = row(r);
            uint8_t* out = &o[(size_t)r * ow];
            if (fancy && dw > 2) {   // h2v1_fancy_upsample
                int inv = in[0];
                out[0] = (uint8_t)inv;
                out[1] = (uint8_t)((inv * 3 + in[1] + 2) >> 2);
                for (int x = 1; x < dw - 1; ++x) {
                    inv = in[x] * 3;
                    out[2 * x] = (uint8_t)((inv + in[x - 1] + 1) >> 2);
                    out[2 * x + 1] = (uint8_t)((inv + in[x + 1] + 2) >> 2);
                }
                inv = in[dw - 1];
                out[2 * dw - 2] = (uint8_t)((inv * 3 + in[dw - 2] + 1) >> 2);
                out[2 * dw - 1] = (uint8_t)inv;
            } else {
                for (int x = 0; x < dw; ++x) out[2 * x] = out[2 * x + 1] = in[x];
            }
        }
    } else if (hx == 1 && vx == 2 && fancy) {   // h1v2_fancy_upsample
        for (int r = 0; r < dh; ++r)
            for (int v = 0; v < 2; ++v) {
                const uint8_t* in0 = row(r);
                const uint8_t* in1 = row(v == 0 ? r - 1 : r + 1);
                const int bias = v == 0 ? 1 : 2;
                uint8_t* out = &o[(size_t)(2 * r + v) * ow];
                for (int x = 0; x < dw; ++x) out[x] = (uint8_t)((in0[x] * 3 + in1[x] + bias) >> 2);
            }
    } else if (hx == 2 && vx == 2 && fancy && dw > 2) {   // h2v2_fancy_upsample
        for (int r = 0; r < dh; ++r)
            for (int v = 0; v < 2; ++v) {
                const uint8_t* in0 = row(r);
                const uint8_t* in1 = row(v == 0 ? r - 1 : r + 1);
                uint8_t* out = &o[(size_t)(2 * r + v) * ow];
                int thiss = in0[0] * 3 + in1[0];
                int next = in0[1] * 3 + in1[1];
                out[0] = (uint8_t)((thiss * 4 + 8) >> 4);
                out[1] = (uint8_t)((thiss * 3 + next + 7) >> 4);
                int last = thiss;
                thiss = next;
                for (int x = 1; x < dw - 1; ++x) {
                    next = in0[x + 1] * 3 + in1[x + 1];
                    out[2 * x] = (uint8_t)((thiss * 3 + last + 8) >> 4);
                    out[2 * x + 1] = (uint8_t)((thiss * 3 + next + 7) >> 4);
                    last = thiss;
                    thiss = next;
                }
                out[2 * dw - 2] = (uint8_t)((thiss * 3 + last + 8) >> 4);
                out[2 * dw - 1] = (uint8_t)((thiss * 4 + 7) >> 4);
            }
    } else {   // h2v2_upsample / int_upsample: box replication
        for (int r = 0; r < oh; ++r) {
            const uint8_t* in = row(r / vx);
            uint8_t* out = &o[(size_t)r * ow];
            for (int x = 0; x < ow; ++x) out[x] = in[x / hx];
        }
    }
    return o;
}

// jdcolor.c build_ycc_rgb_table (SCALEBITS 16)
struct YccTables {
    int cr_r[256], cb_b[256];
    int64_t cr_g[256], cb_g[256];
    YccTables() {
        constexpr int64_t ONE_HALF = (int64_t)1 << 15;
        auto fix = [](double x) { return (int64_t)(x * 65536.0 + 0.5); };
        for (int i = 0; i < 256; ++i) {
            const int64_t x = i - 128;
            cr_r[i] = (int)((fix(1.40200) * x + ONE_HALF) >> 16);
            cb_b[i] = (int)((fix(1.77200) * x + ONE_HALF) >> 16);
            cr_g[i] = -fix(0.71414) * x;
            cb_g[i] = -fix(0.34414) * x + ONE_HALF;
        }
    }
};
const YccTables kYcc;
inline uint8_t clamp255(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

uint16_t be16(const uint8_t* p) { return (uint16_t)(p[0] << 8 | p[1]); }

// EXIF orientation (tag 0x0112 of IFD0 in an APP1 "Exif\0\0" segment, TIFF byte order "II" / "MM");
// 1 when absent or unreadable.  cv::imread(IMREAD_COLOR) applies it (OpenCV's ExifTransform).
int exif_orientation(const uint8_t* b, int n) {
    if (n < 14 || std::memcmp(b, "Exif\0\0", 6) != 0) return 1;
    const uint8_t* t = b + 6;
    const int64_t tn = n - 6;
    bool le;
    if (t[0] == 'I' && t[1] == 'I') le = true;
    else if (t[0] == 'M' && t[1] == 'M') le = false;
    else return 1;
    auto u16 = [&](int64_t o) -> uint32_t { return le ? (uint32_t)(t[o] | t[o + 1] << 8) : (uint32_t)(t[o] << 8 | t[o + 1]); };
    auto u32 = [&](int64_t o) -> uint32_t {
        return le ? (uint32_t)t[o] | (uint32_t)t[o + 1] << 8 | (uint32_t)t[o + 2] << 16 | (uint32_t)t[o + 3] << 24
                  : (uint32_t)t[o] << 24 | (uint32_t)t[o + 1] << 16 | (uint32_t)t[o + 2] << 8 | (uint32_t)t[o + 3];
    };
    if (u16(2) != 42) return 1;
    const int64_t ifd = u32(4);
    if (ifd + 2 > tn) return 1;
    const int64_t cnt = u16(ifd);
    for (int64_t i = 0; i < cnt; ++i) {
        const int64_t e = ifd + 2 + 12 * i;
        if (e + 12 > tn) return 1;
        if (u16(e) == 0x0112) {
            if (u16(e + 2) != 3) return 1;   // SHORT
            const uint32_t v = u16(e + 8);
            return v >= 1 && v <= 8 ? (int)v : 1;
        }
    }
    return 1;
}

// the EXIF orientation transform of an (h, w, c) image, as OpenCV's ExifTransform applies it:
// 2 flip left-right, 3 rotate 180, 4 flip top-bottom, 5 transpose, 6 rotate 90 clockwise,
// 7 transverse (transpose + rotate 180), 8 rotate 90 counter-clockwise
void apply_orientation(Decoded& d, int o) {
    if (o <= 1) return;
    const int h = d.h, w = d.w, c = d.c;
    const bool swap = o >= 5;
    const int oh = swap ? w : h, ow = swap ? h : w;
    std::vector<uint8_t> px((size_t)oh * ow * c);
    for (int y = 0; y < oh; ++y)
        for (int x = 0; x < ow; ++x) {
            int sy, sx;   // source pixel of output (y, x)
            switch (o) {
                case 2: sy = y; sx = w - 1 - x; break;
                case 3: sy = h - 1 - y; sx = w - 1 - x; break;
                case 4: sy = h - 1 - y; sx = x; break;
                case 5: sy = x; sx = y; break;
                case 6: sy = h - 1 - x; sx = y; break;
                case 7: sy = h - 1 - x; sx = w - 1 - y; break;
                default: sy = x; sx = w - 1 - y; break;   // 8
            }
            std::memcpy(&px[((size_t)y * ow + x) * c], &d.px[((size_t)sy * w + sx) * c], (size_t)c);
        }
    d.px.swap(px);
    d.h = oh;
    d.w = ow;
}

}  // namespace

Decoded decode(const uint8_t* data, size_t size) {
    if (size < 4 || data[0] != 0xFF || data[1] != 0xD8) throw JpegError("not a JPEG file (no SOI marker)");
    const uint8_t* p = data + 2;
    const uint8_t* end = data + size;
    int16_t qt[4][64];
    bool qdef[4] = {false, false, false, false};
    Huffman dc[4], ac[4];
    std::vector<Component> comps;
    int W = 0, H = 0, hmax = 1, vmax = 1, restart = 0;
    bool jfif = false, adobe = false, frame = false, any_scan = false, progressive = false;
    int adobe_transform = -1, orientation = 1;

    auto seg = [&](const uint8_t*& q) -> std::pair<const uint8_t*, int> {
        if (q + 2 > end) throw JpegError("truncated marker segment");
        const int len = be16(q);
        if (len < 2 || q + len > end) throw JpegError("bad marker segment length");
        const uint8_t* body = q + 2;
        q += len;
        return {body, len - 2};
    };

    for (;;) {
        // next marker (fill bytes 0xFF allowed)
        while (p < end && *p != 0xFF) ++p;
        while (p < end && *p == 0xFF) ++p;
        if (p >= end) throw JpegError("premature end of JPEG file");
        const int m = *p++;
        if (m == 0xD9) break;                                  // EOI
        if (m >= 0xD0 && m <= 0xD7) continue;                 // stray RSTn
        if (m == 0x01) continue;                              // TEM
        auto [b, n] = seg(p);
        if (m == 0xC4) {                                      // DHT
            int k = 0;
            while (k < n) {
                if (k + 17 > n) throw JpegError("truncated DHT");
                const int tc = b[k] >> 4, th = b[k] & 15;
                if (tc > 1 || th > 3) throw JpegError("bad DHT table id");
                uint8_t bits[17] = {0};
                int total = 0;
                for (int l = 1; l <= 16; ++l) total += bits[l] = b[k + l];
                if (total > 256 || k + 17 + total > n) throw JpegError("bad DHT counts");
                (tc ? ac[th] : dc[th]).build(bits, b + k + 17, total, tc == 0);
                k += 17 + total;
            }
        } else if (m == 0xDB) {                               // DQT
            int k = 0;
            while (k < n) {
                const int pq = b[k] >> 4, tq = b[k] & 15;
                if (tq > 3 || pq > 1) throw JpegError("bad DQT table id");
                if (k + 1 + 64 * (pq + 1) > n) throw JpegError("truncated DQT");
                for (int i = 0; i < 64; ++i)
                    qt[tq][kNatural[i]] = (int16_t)(pq ? be16(b + k + 1 + 2 * i) : b[k + 1 + i]);
                qdef[tq] = true;
                k += 1 + 64 * (pq + 1);
            }
        } else if (m == 0xDD) {                               // DRI
            if (n < 2) throw JpegError("bad DRI");
            restart = be16(b);
        } else if (m == 0xE0) {                               // APP0
            if (n >= 5 && std::memcmp(b, "JFIF\0", 5) == 0) jfif = true;
        } else if (m == 0xE1) {                               // APP1 (EXIF orientation)
            if (orientation == 1) orientation = exif_orientation(b, n);
        } else if (m == 0xEE) {                               // APP14
            if (n >= 12 && std::memcmp(b, "Adobe", 5) == 0) {
                adobe = true;
                adobe_transform = b[11];
            }
        } else if (m == 0xC0 || m == 0xC1 || m == 0xC2) {     // SOF0 / SOF1: sequential, SOF2: progressive Huffman
            if (frame) throw JpegError("more than one frame");
            progressive = m == 0xC2;
            if (n < 6 || b[0] != 8) throw JpegError("only 8-bit JPEG samples are supported");
            H = be16(b + 1);
            W = be16(b + 3);
            const int nc = b[5];
            if (W <= 0 || H <= 0) throw JpegError("bad image size (DNL not supported)");
            if ((nc != 1 && nc != 3) || n < 6 + 3 * nc) throw JpegError("only 1- and 3-component JPEGs are supported");
            comps.resize((size_t)nc);
            for (int i = 0; i < nc; ++i) {
                Component& c = comps[(size_t)i];
                c.id = b[6 + 3 * i];
                c.h = b[7 + 3 * i] >> 4;
                c.v = b[7 + 3 * i] & 15;
                c.tq = b[8 + 3 * i];
                if (c.h < 1 || c.h > 4 || c.v < 1 || c.v > 4 || c.tq > 3) throw JpegError("bad sampling factors");
                hmax = std::max(hmax, c.h);
                vmax = std::max(vmax, c.v);
            }
            const int mcux = (W + 8 * hmax - 1) / (8 * hmax), mcuy = (H + 8 * vmax - 1) / (8 * vmax);
            for (Component& c : comps) {
                c.bw = mcux * c.h;
                c.bh = mcuy * c.v;
                c.dw = (int)(((int64_t)W * c.h + hmax - 1) / hmax);
                c.dh = (int)(((int64_t)H * c.v + vmax - 1) / vmax);
                c.coef.assign((size_t)c.bw * c.bh * 64, 0);
                std::fill(c.coef_bits, c.coef_bits + 64, -1);
            }
            frame = true;
        } else if (m == 0xC6 || m == 0xCA || m == 0xCE) {
            throw JpegError("differential / arithmetic-coded progressive JPEG is not supported");
        } else if (m == 0xC3 || m == 0xC7 || m == 0xCB || m == 0xCF) {
            throw JpegError("lossless JPEG is not supported");
        } else if (m == 0xC9 || m == 0xCA || m == 0xCB || m == 0xCD) {
            throw JpegError("arithmetic-coded JPEG is not supported");
        } else if (m == 0xC5) {
            throw JpegError("hierarchical JPEG is not supported");
        } else if (m == 0xDA) {                               // SOS
            if (!frame) throw JpegError("scan before frame header");
            const int ns = n > 0 ? b[0] : 0;
            if (ns < 1 || ns > 4 || n < 4 + 2 * ns) throw JpegError("bad SOS");
            std::vector<Component*> sc;
            for (int i = 0; i < ns; ++i) {
                Component* c = nullptr;
                for (Component& x : comps)
                    if (x.id == b[1 + 2 * i]) c = &x;
                if (!c) throw JpegError("SOS names an unknown component");
                c->td = b[2 + 2 * i] >> 4;
                c->ta = b[2 + 2 * i] & 15;
                if (c->td > 3 || c->ta > 3) throw JpegError("scan uses an undefined Huffman table");
                sc.push_back(c);
            }
            const int ss = b[1 + 2 * ns], se = b[2 + 2 * ns], ah = b[3 + 2 * ns] >> 4, al = b[3 + 2 * ns] & 15;
            // the Huffman tables the scan decodes with: sequential DC + AC, progressive DC first (DC
            // tables), AC scans (AC tables), DC refinement (none)
            const bool need_dc = !progressive || (ss == 0 && ah == 0), need_ac = !progressive || ss > 0;
            for (Component* c : sc)
                if ((need_dc && !dc[c->td].defined) || (need_ac && !ac[c->ta].defined))
                    throw JpegError("scan uses an undefined Huffman table");
            if (!progressive) {
                if (ss != 0 || se != 63 || ah != 0 || al != 0) throw JpegError("not a sequential scan");
            } else {   // jdphuff.c start_pass_phuff_decoder's JERR_BAD_PROGRESSION checks
                const bool bad = (ss == 0 ? se != 0 : (ss > se || se > 63 || ns != 1)) ||
                                 (ah != 0 && al != ah - 1) || al > 13;
                if (bad) throw JpegError("bad progressive scan parameters");
                for (Component* c : sc)
                    for (int k = ss; k <= se; ++k) c->coef_bits[k] = al;
            }
            for (Component* c : sc) c->pred = 0;
            int eobrun = 0;
            // entropy-coded segment
            Bits bits{p, end};
            int mx, my;
            if (ns == 1) {   // non-interleaved: the component's own blocks covering its samples
                mx = (sc[0]->dw + 7) / 8;
                my = (sc[0]->dh + 7) / 8;
            } else {
                mx = (W + 8 * hmax - 1) / (8 * hmax);
                my = (H + 8 * vmax - 1) / (8 * vmax);
            }
            const int64_t total = (int64_t)mx * my;
            int todo = restart;
            for (int64_t u = 0; u < total; ++u) {
                if (restart && todo == 0) {   // expect RSTn: drop the partial byte, skip the marker
                    bits.reset();
                    const uint8_t* q = bits.p;
                    while (q < end && *q != 0xFF) ++q;
                    while (q < end && *q == 0xFF) ++q;
                    if (q < end && *q >= 0xD0 && *q <= 0xD7) ++q;
                    bits.p = q;
                    bits.at_marker = false;
                    for (Component* c : sc) c->pred = 0;
                    eobrun = 0;
                    todo = restart;
                }
                const int ux = (int)(u % mx), uy = (int)(u / mx);
                for (Component* c : sc) {
                    const int nbx = ns == 1 ? 1 : c->h, nby = ns == 1 ? 1 : c->v;
                    for (int by = 0; by < nby; ++by)
                        for (int bx = 0; bx < nbx; ++bx) {
                            const int gx = ux * nbx + bx, gy = uy * nby + by;
                            int16_t* blk = &c->coef[((size_t)gy * c->bw + gx) * 64];
                            if (progressive) {
                                if (ss == 0) {
                                    if (ah == 0) dc_first(bits, dc[c->td], *c, al, blk);
                                    else dc_refine(bits, al, blk);
                                } else if (ah == 0) {
                                    ac_first(bits, ac[c->ta], ss, se, al, eobrun, blk);
                                } else {
                                    ac_refine(bits, ac[c->ta], ss, se, al, eobrun, blk);
                                }
                                continue;
                            }
                            const int t = bits.decode(dc[c->td]);
                            if (t > 11) throw JpegError("bad DC coefficient");
                            const int diff = t ? extend(bits.get(t), t) : 0;
                            c->pred += diff;
                            blk[0] = (int16_t)c->pred;
                            for (int k = 1; k < 64; ++k) {
                                const int rs = bits.decode(ac[c->ta]);
                                const int r = rs >> 4, s = rs & 15;
                                if (s) {
                                    k += r;
                                    blk[kNatural[k]] = (int16_t)extend(bits.get(s), s);
                                } else {
                                    if (r != 15) break;
                                    k += 15;
                                }
                            }
                        }
                }
                if (restart) --todo;
            }
            // resume marker parsing at the end of the entropy-coded data
            const uint8_t* q = bits.p;
            while (q + 1 < end && !(q[0] == 0xFF && q[1] != 0x00 && !(q[1] >= 0xD0 && q[1] <= 0xD7))) ++q;
            p = q;
            any_scan = true;
        } else if (m == 0xC8 || (m >= 0xF0 && m <= 0xFD) || m == 0xDC || m == 0xDE || m == 0xDF) {
            // JPG extensions / DNL / DHP / EXP: ignored (as libjpeg skips unknown segments)
        }
        // APPn (other), COM: skipped
    }
    if (!frame || !any_scan) throw JpegError("JPEG file has no image data");
    if (progressive)   // libjpeg-turbo's output pass would smooth these blocks (jdcoefct.c smoothing_ok)
        for (const Component& c : comps) {
            if (c.coef_bits[0] < 0) continue;   // no DC scan: no smoothing either
            for (int k = 1; k < 10; ++k)
                if (c.coef_bits[k] != 0)
                    throw JpegError("progressive JPEG with incompletely refined coefficients (block smoothing) "
                                    "is not supported");
        }

    // dequantise + inverse DCT every block of every component
    for (Component& c : comps) {
        if (!qdef[c.tq]) throw JpegError("undefined quantisation table");
        c.plane.assign((size_t)c.bw * 8 * c.bh * 8, 0);
        const int ls = c.bw * 8;
        for (int by = 0; by < c.bh; ++by)
            for (int bx = 0; bx < c.bw; ++bx)
                idct_islow(&c.coef[((size_t)by * c.bw + bx) * 64], qt[c.tq], &c.plane[(size_t)by * 8 * ls + bx * 8], ls);
        std::vector<int16_t>().swap(c.coef);
    }
    Decoded out;
    out.h = H;
    out.w = W;
    const bool fancy = true;   // do_fancy_upsampling default (min_DCT_scaled_size 8 > 1)
    if (comps.size() == 1) {
        out.c = 1;
        out.px.resize((size_t)W * H);
        const Component& c = comps[0];
        for (int r = 0; r < H; ++r) std::memcpy(&out.px[(size_t)r * W], &c.plane[(size_t)r * c.bw * 8], (size_t)W);
        apply_orientation(out, orientation);
        return out;
    }
    // colour space (jdapimin.c default_decompress_parms): JFIF -> YCbCr; Adobe transform 0 -> RGB;
    // otherwise component ids 'R','G','B' -> RGB, anything else YCbCr
    bool ycc = true;
    if (jfif) ycc = true;
    else if (adobe) ycc = adobe_transform != 0;
    else if (comps[0].id == 82 && comps[1].id == 71 && comps[2].id == 66) ycc = false;
    std::vector<uint8_t> up[3];
    int uw[3];
    for (int i = 0; i < 3; ++i) {
        const Component& c = comps[(size_t)i];
        if (hmax % c.h || vmax % c.v) throw JpegError("fractional sampling factors are not supported");
        up[i] = upsample(c, hmax / c.h, vmax / c.v, fancy);
        uw[i] = c.dw * (hmax / c.h);
    }
    out.c = 3;
    out.px.resize((size_t)W * H * 3);
    for (int r = 0; r < H; ++r) {
        const uint8_t* y = &up[0][(size_t)r * uw[0]];
        const uint8_t* cb = &up[1][(size_t)r * uw[1]];
        const uint8_t* cr = &up[2][(size_t)r * uw[2]];
        uint8_t* o = &out.px[(size_t)r * W * 3];
        for (int x = 0; x < W; ++x) {
            if (ycc) {
                const int Y = y[x];
                o[3 * x + 0] = clamp255(Y + kYcc.cr_r[cr[x]]);
                o[3 * x + 1] = clamp255(Y + (int)((kYcc.cb_g[cb[x]] + kYcc.cr_g[cr[x]]) >> 16));
                o[3 * x + 2] = clamp255(Y + kYcc.cb_b[cb[x]]);
            } else {
                o[3 * x + 0] = y[x];
                o[3 * x + 1] = cb[x];
                o[3 * x + 2] = cr[x];
            }
        }
    }
    apply_orientation(out, orientation);
    return out;
}

}  // namespace jpeg
}  // namespace cad
