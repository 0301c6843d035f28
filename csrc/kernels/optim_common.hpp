// Fused DiLoCo outer-step math shared by the host loop and the HIP kernel (one definition, -ffp-contract=off on both).
//
// DiLoCo (reference python/examples/nanogpt_diloco/sync_diloco.py:280-330) keeps fp32 "outer" parameters, computes
// the pseudo-gradient  g = outer - local  after H inner steps, averages g over all peers, then applies an SGD step
// with (Nesterov) momentum to the outer parameters and copies them back into the model. Unfused this is ~5 passes
// over the parameters (sub, mul_/add_ momentum, add_ nesterov, add_ update, copy_); fused it is one pass:
//
//   g' = g + wd * outer
//   m  = first ? g' : momentum * m + (1 - dampening) * g'
//   d  = nesterov ? g' + momentum * m : m
//   outer = outer - lr * d ;  local = cast(outer)
//
// which is torch.optim.SGD's update rule (momentum buffer initialised to the first gradient).
#pragma once

#include <cstddef>
#include <cstdint>

#include "../common/numeric.hpp"

namespace pccl::kernels {

struct OuterSgdParams {
    float lr = 0.7f;
    float momentum = 0.9f;
    float dampening = 0.0f;
    float weight_decay = 0.0f;
    int nesterov = 1;
    int first = 0; // first outer step: momentum buffer := gradient
};

PCCL_HD void outer_sgd_elem(float &outer, float &mom, float g, const OuterSgdParams &p) {
    if (p.weight_decay != 0.0f) g = g + p.weight_decay * outer;
    float m;
    if (p.first) {
        m = g;
    } else {
        const float a = p.momentum * mom;
        const float b = (1.0f - p.dampening) * g;
        m = a + b;
    }
    mom = m;
    float d = m;
    if (p.nesterov) {
        const float c = p.momentum * m;
        d = g + c;
    }
    const float u = p.lr * d;
    outer = outer - u;
}

} // namespace pccl::kernels
