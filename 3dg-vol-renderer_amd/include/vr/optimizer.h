// optimizer.h — C++ mirror of the reference's include/optimizer.h over the C ABI (include/vr_hip.h).
#pragma once
#include "gmm.h"
// optimizer.h:13-55 — AdamOptimizer (the step is vr_adam_step)
class AdamOptimizer {
public:
    AdamOptimizer(size_t ndim, float lr = 1e-3f, float beta1 = 0.9f, float beta2 = 0.999f, float eps = 1e-8f)
        : m(ndim, 0.0f), v(ndim, 0.0f), lr(lr), beta1(beta1), beta2(beta2), eps(eps), t(0) {}
    bool step(std::vector<float>& params, const std::vector<float>& grads) {
        if (params.size() != grads.size() || params.size() != m.size() || params.size() != v.size()) return false;
        ++t;
        vr_cpp::check(vr_adam_step(params.data(), grads.data(), m.data(), v.data(), params.size(), t, lr, beta1, beta2, eps));
        return true;
    }
    void reset_state() {
        std::fill(m.begin(), m.end(), 0.0f);
        std::fill(v.begin(), v.end(), 0.0f);
        t = 0;
    }
    size_t dim() const { return m.size(); }

private:
    std::vector<float> m, v;
    float lr, beta1, beta2, eps;
    int t;
};

