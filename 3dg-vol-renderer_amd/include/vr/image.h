// image.h — C++ mirror of the reference's include/image.h over the C ABI (include/vr_hip.h).
#pragma once
#include "runtime.h"
// ---------------------------------------------------------------------------------------------
// image.h:9-106
// ---------------------------------------------------------------------------------------------
class Image {
    unsigned int width = 0, height = 0;
    std::vector<float> pixels;

public:
    Image(unsigned int w, unsigned int h) : width(w), height(h), pixels(3 * (size_t)w * h, 0.0f) {}
    explicit Image(const std::string& filename) {
        vr_cpp::check(vr_image_read_ppm(filename.c_str(), nullptr, &width, &height));
        pixels.resize(3 * (size_t)width * height);
        vr_cpp::check(vr_image_read_ppm(filename.c_str(), pixels.data(), &width, &height));
    }
    unsigned int get_width() const { return width; }
    unsigned int get_height() const { return height; }
    Eigen::Vector3f get_pixel(unsigned i, unsigned j) const {
        size_t k = 3 * ((size_t)j * width + i);
        return Eigen::Vector3f(pixels[k], pixels[k + 1], pixels[k + 2]);
    }
    void set_pixel(unsigned i, unsigned j, const Eigen::Vector3f& rgb) {
        size_t k = 3 * ((size_t)j * width + i);
        pixels[k] = rgb[0];
        pixels[k + 1] = rgb[1];
        pixels[k + 2] = rgb[2];
    }
    void make_PPM(const std::string& filename) const {
        vr_cpp::check(vr_image_write_ppm(filename.c_str(), pixels.data(), width, height));
    }
    std::vector<uint8_t> get_rgba_buffer() const {
        std::vector<uint8_t> buf(4 * (size_t)width * height);
        for (size_t p = 0; p < (size_t)width * height; ++p) {
            for (int c = 0; c < 3; ++c)
                buf[4 * p + c] = static_cast<uint8_t>(std::clamp(pixels[3 * p + c] * 255.0f, 0.0f, 255.0f));
            buf[4 * p + 3] = 255;
        }
        return buf;
    }
    float* data() { return pixels.data(); }
    const float* data() const { return pixels.data(); }
};

