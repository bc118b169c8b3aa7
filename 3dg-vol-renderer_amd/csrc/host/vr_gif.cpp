// Animated GIF writer for the turntable mode of the reference driver (tests/main.cpp:81-114, which
// uses gif-h's GifBegin / GifWriteFrame / GifEnd; gif-h is an empty submodule in the reference, so
// this is an independent GIF89a encoder with the same role):
//   * every frame gets its own 256-colour palette: median cut over the frame's colours, histogrammed
//     at 5 bits per channel, then nearest-palette-entry mapping through a 32768-entry table;
//   * LZW-compressed image data (variable code width from 9 bits, clear code at 4096 entries);
//   * NETSCAPE2.0 looping extension and a per-frame delay in hundredths of a second.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "vr_common.h"

using namespace vr;

struct vr_gif {
    FILE* f = nullptr;
    uint32_t w = 0, h = 0, delay = 0;
};

namespace {

void put16(FILE* f, uint32_t v) {
    std::fputc((int)(v & 0xff), f);
    std::fputc((int)((v >> 8) & 0xff), f);
}

// Median cut over the 5-bit histogram: split the box with the most pixels along its longest axis
// at the pixel median until there are 256 boxes; each palette entry is its box's mean colour.
void median_cut(const std::vector<uint32_t>& hist, uint8_t pal[256][3], std::vector<uint8_t>& lut) {
    struct Box { int lo[3], hi[3]; uint64_t n; };
    auto count = [&](const Box& b) {
        uint64_t n = 0;
        for (int r = b.lo[0]; r <= b.hi[0]; ++r)
            for (int g = b.lo[1]; g <= b.hi[1]; ++g)
                for (int c = b.lo[2]; c <= b.hi[2]; ++c) n += hist[(r << 10) | (g << 5) | c];
        return n;
    };
    std::vector<Box> boxes{{{0, 0, 0}, {31, 31, 31}, 0}};
    boxes[0].n = count(boxes[0]);
    while (boxes.size() < 256) {
        int bi = -1;
        uint64_t best = 0;
        for (size_t i = 0; i < boxes.size(); ++i) {
            const Box& b = boxes[i];
            const bool splittable = b.hi[0] > b.lo[0] || b.hi[1] > b.lo[1] || b.hi[2] > b.lo[2];
            if (splittable && b.n > best) {
                best = b.n;
                bi = (int)i;
            }
        }
        if (bi < 0) break;
        Box b = boxes[bi];
        int ax = 0;
        for (int k = 1; k < 3; ++k)
            if (b.hi[k] - b.lo[k] > b.hi[ax] - b.lo[ax]) ax = k;
        // pixel median along ax
        std::vector<uint64_t> slab(32, 0);
        for (int r = b.lo[0]; r <= b.hi[0]; ++r)
            for (int g = b.lo[1]; g <= b.hi[1]; ++g)
                for (int c = b.lo[2]; c <= b.hi[2]; ++c) {
                    const int v[3] = {r, g, c};
                    slab[v[ax]] += hist[(r << 10) | (g << 5) | c];
                }
        uint64_t acc = 0;
        int cut = b.lo[ax];
        for (int v = b.lo[ax]; v < b.hi[ax]; ++v) {
            acc += slab[v];
            cut = v;
            if (2 * acc >= b.n) break;
        }
        Box l = b, r = b;
        l.hi[ax] = cut;
        r.lo[ax] = cut + 1;
        l.n = count(l);
        r.n = b.n - l.n;
        boxes[bi] = l;
        boxes.push_back(r);
    }
    lut.assign(32768, 0);
    for (size_t i = 0; i < 256; ++i) {
        if (i >= boxes.size()) {
            pal[i][0] = pal[i][1] = pal[i][2] = 0;
            continue;
        }
        const Box& b = boxes[i];
        double s[3] = {0, 0, 0};
        uint64_t n = 0;
        for (int r = b.lo[0]; r <= b.hi[0]; ++r)
            for (int g = b.lo[1]; g <= b.hi[1]; ++g)
                for (int c = b.lo[2]; c <= b.hi[2]; ++c) {
                    const uint32_t k = (r << 10) | (g << 5) | c;
                    const double m = hist[k];
                    s[0] += m * (r * 8 + 4);
                    s[1] += m * (g * 8 + 4);
                    s[2] += m * (c * 8 + 4);
                    n += hist[k];
                }
        for (int k = 0; k < 3; ++k)
            pal[i][k] = (uint8_t)std::clamp(n ? s[k] / (double)n : (b.lo[k] + b.hi[k]) * 4.0 + 4.0, 0.0, 255.0);
    }
    for (uint32_t k = 0; k < 32768; ++k) {  // nearest entry for every 5-bit colour
        const int r = (int)(k >> 10) * 8 + 4, g = (int)((k >> 5) & 31) * 8 + 4, c = (int)(k & 31) * 8 + 4;
        int best = 0, bd = 1 << 30;
        for (size_t i = 0; i < std::min<size_t>(256, boxes.size()); ++i) {
            const int dr = r - pal[i][0], dg = g - pal[i][1], db = c - pal[i][2];
            const int d = dr * dr + dg * dg + db * db;
            if (d < bd) {
                bd = d;
                best = (int)i;
            }
        }
        lut[k] = (uint8_t)best;
    }
}

// GIF LZW (8-bit indices): codes packed LSB-first into 255-byte sub-blocks.
void lzw_write(FILE* f, const std::vector<uint8_t>& idx) {
    const int min_bits = 8, clear = 1 << min_bits, eoi = clear + 1;
    std::fputc(min_bits, f);
    std::vector<uint8_t> block;
    uint32_t bitbuf = 0;
    int nbits = 0, width = min_bits + 1;
    auto flush_block = [&](bool all) {
        while (block.size() >= 255 || (all && !block.empty())) {
            const size_t n = std::min<size_t>(255, block.size());
            std::fputc((int)n, f);
            std::fwrite(block.data(), 1, n, f);
            block.erase(block.begin(), block.begin() + n);
        }
    };
    auto emit = [&](int code) {
        bitbuf |= (uint32_t)code << nbits;
        nbits += width;
        while (nbits >= 8) {
            block.push_back((uint8_t)(bitbuf & 0xff));
            bitbuf >>= 8;
            nbits -= 8;
        }
        if (block.size() >= 255) flush_block(false);
    };
    // dictionary: (prefix code, byte) -> code, as a 4096 x 256 table of next codes
    std::vector<int16_t> next(4096 * 256, -1);
    int next_code = eoi + 1;
    emit(clear);
    if (!idx.empty()) {
        int cur = idx[0];
        for (size_t i = 1; i < idx.size(); ++i) {
            const int c = idx[i];
            const int16_t n = next[(size_t)cur * 256 + c];
            if (n >= 0) {
                cur = n;
                continue;
            }
            emit(cur);
            if (next_code < 4096) {  // new entry. The decoder adds each entry one code later than the
                // encoder and widens once its table reaches 2^width, so the encoder widens when the entry
                // it adds is number 2^width itself.
                next[(size_t)cur * 256 + c] = (int16_t)next_code;
                if (next_code == (1 << width) && width < 12) ++width;
                ++next_code;
            }
            if (next_code >= 4096) {  // table full: clear and restart at 9-bit codes
                emit(clear);
                std::fill(next.begin(), next.end(), (int16_t)-1);
                next_code = eoi + 1;
                width = min_bits + 1;
            }
            cur = c;
        }
        emit(cur);
    }
    emit(eoi);
    if (nbits > 0) block.push_back((uint8_t)(bitbuf & 0xff));
    flush_block(true);
    std::fputc(0, f);  // block terminator
}

}  // namespace

extern "C" {

vr_status vr_gif_begin(const char* path, uint32_t width, uint32_t height, uint32_t delay_cs, vr_gif** out) {
    if (!path || !out || width == 0 || height == 0 || width > 65535 || height > 65535)
        return fail(VR_ERR_INVALID, "vr_gif_begin: bad argument");
    FILE* f = std::fopen(path, "wb");
    if (!f) return fail(VR_ERR_IO, std::string("cannot open ") + path);
    auto* g = new vr_gif();
    g->f = f;
    g->w = width;
    g->h = height;
    g->delay = delay_cs;
    std::fwrite("GIF89a", 1, 6, f);
    put16(f, width);
    put16(f, height);
    std::fputc(0x00, f);  // no global colour table (every frame has its own)
    std::fputc(0, f);
    std::fputc(0, f);
    // NETSCAPE2.0: loop forever
    const uint8_t ext[] = {0x21, 0xff, 0x0b, 'N', 'E', 'T', 'S', 'C', 'A', 'P', 'E', '2', '.', '0', 0x03, 0x01, 0x00, 0x00, 0x00};
    std::fwrite(ext, 1, sizeof(ext), f);
    *out = g;
    return VR_OK;
}

vr_status vr_gif_write_frame(vr_gif* g, const uint8_t* rgba, uint32_t delay_cs) {
    if (!g || !g->f || !rgba) return fail(VR_ERR_INVALID, "vr_gif_write_frame: bad argument");
    const size_t npix = (size_t)g->w * g->h;
    std::vector<uint32_t> hist(32768, 0);
    std::vector<uint16_t> key(npix);
    for (size_t p = 0; p < npix; ++p) {
        const uint16_t k = (uint16_t)(((rgba[4 * p] >> 3) << 10) | ((rgba[4 * p + 1] >> 3) << 5) | (rgba[4 * p + 2] >> 3));
        key[p] = k;
        hist[k]++;
    }
    uint8_t pal[256][3];
    std::vector<uint8_t> lut;
    median_cut(hist, pal, lut);
    std::vector<uint8_t> idx(npix);
    for (size_t p = 0; p < npix; ++p) idx[p] = lut[key[p]];
    FILE* f = g->f;
    const uint8_t gce[] = {0x21, 0xf9, 0x04, 0x00, (uint8_t)(delay_cs & 0xff), (uint8_t)((delay_cs >> 8) & 0xff), 0x00, 0x00};
    std::fwrite(gce, 1, sizeof(gce), f);
    std::fputc(0x2c, f);  // image descriptor
    put16(f, 0);
    put16(f, 0);
    put16(f, g->w);
    put16(f, g->h);
    std::fputc(0x87, f);  // local colour table of 2^(7+1) = 256 entries
    std::fwrite(pal, 1, sizeof(pal), f);
    lzw_write(f, idx);
    if (std::ferror(f)) return fail(VR_ERR_IO, "vr_gif_write_frame: write failed");
    return VR_OK;
}

vr_status vr_gif_end(vr_gif* g) {
    if (!g) return fail(VR_ERR_INVALID, "vr_gif_end: NULL");
    vr_status st = VR_OK;
    if (g->f) {
        std::fputc(0x3b, g->f);  // trailer
        if (std::fclose(g->f) != 0) st = fail(VR_ERR_IO, "vr_gif_end: close failed");
    }
    delete g;
    return st;
}

}  // extern "C"
