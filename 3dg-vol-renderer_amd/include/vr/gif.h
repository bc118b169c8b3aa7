// gif.h — the gif-h interface tests/main.cpp:81-114 uses for its turntable (GifBegin / GifWriteFrame /
// GifEnd; gif-h is an empty submodule in the reference), over the library's GIF89a encoder
// (vr_gif_*: per-frame 256-colour median-cut palette, LZW, looping). bitDepth / dither are accepted
// for signature compatibility; frames are always 8-bit palettes without dithering.
#pragma once
#include "runtime.h"

struct GifWriter {
    vr_gif* g = nullptr;
    uint32_t width = 0, height = 0;
};

inline bool GifBegin(GifWriter* w, const char* filename, uint32_t width, uint32_t height, uint32_t delay,
                     int32_t bitDepth = 8, bool dither = false) {
    (void)bitDepth;
    (void)dither;
    if (!w || vr_gif_begin(filename, width, height, delay, &w->g) != VR_OK) return false;
    w->width = width;
    w->height = height;
    return true;
}

inline bool GifWriteFrame(GifWriter* w, const uint8_t* image, uint32_t width, uint32_t height, uint32_t delay,
                          int bitDepth = 8, bool dither = false) {
    (void)bitDepth;
    (void)dither;
    if (!w || !w->g || width != w->width || height != w->height) return false;
    return vr_gif_write_frame(w->g, image, delay) == VR_OK;
}

inline bool GifEnd(GifWriter* w) {
    if (!w || !w->g) return false;
    const bool ok = vr_gif_end(w->g) == VR_OK;
    w->g = nullptr;
    return ok;
}
