// Runtime of the C++ mirror: status checks (std::runtime_error, the reference's error convention) and the
// device contexts the integrators render on (one per GPU, or a multi-GPU group, vr_init_multi).
#pragma once
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/vr_hip.h"
#include "linalg.h"

namespace vr_cpp {

inline void check(vr_status st) {
    if (st != VR_OK) throw std::runtime_error(vr_last_error());
}

// One device context per GPU, created on first use (vr_init), destroyed at exit.
inline vr_ctx* device(int dev = 0) {
    static std::mutex mu;
    static std::vector<std::unique_ptr<vr_ctx, void (*)(vr_ctx*)>> ctxs;
    std::lock_guard<std::mutex> lock(mu);
    while ((int)ctxs.size() <= dev) ctxs.emplace_back(nullptr, &vr_destroy);
    if (!ctxs[dev]) {
        vr_ctx* c = nullptr;
        check(vr_init(dev, &c));
        ctxs[dev].reset(c);
    }
    return ctxs[dev].get();
}

// Number of visible GPUs.
inline int device_count() {
    int32_t n = 0;
    check(vr_device_count(&n));
    return n;
}

// One multi-GPU context per device list (vr_init_multi), created on first use.
inline vr_ctx* device_group(const std::vector<int>& devs) {
    static std::mutex mu;
    static std::map<std::vector<int>, std::unique_ptr<vr_ctx, void (*)(vr_ctx*)>> groups;
    std::lock_guard<std::mutex> lock(mu);
    auto it = groups.find(devs);
    if (it == groups.end()) {
        std::vector<int32_t> d(devs.begin(), devs.end());
        vr_ctx* c = nullptr;
        check(vr_init_multi((int32_t)d.size(), d.data(), &c));
        it = groups.emplace(devs, std::unique_ptr<vr_ctx, void (*)(vr_ctx*)>(c, &vr_destroy)).first;
    }
    return it->second.get();
}

inline uint64_t next_serial() {
    static std::atomic<uint64_t> serial{0};
    return ++serial;
}

inline uint64_t fnv1a(const void* p, size_t n, uint64_t h = 1469598103934665603ull) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}

}  // namespace vr_cpp
