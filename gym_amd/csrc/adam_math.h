// Adam/AdamW element update shared by the inner-optimizer kernel (optim.hip) and
// the replica loop's fused AdamW + SPARTA step (sparta.hip), so both compute the
// same bits.  Per element (f32 arena, f32 state), in torch's op order
// (torch/optim/adam.py _multi_tensor_adam):
//   p *= 1 - lr*wd                              (AdamW: decoupled decay)   | g += wd*p (Adam: L2)
//   m  = lerp(m, g, 1-b1)                       (torch's lerp: m + w*(g-m) for w < 0.5)
//   v  = b2*v + (1-b2)*g*g
//   p += step_size * m / (sqrt(v)/bc2_sqrt + eps),  step_size = -lr/(1-b1^t), bc2_sqrt = sqrt(1-b2^t)
#pragma once

namespace ga {

struct AdamParams {
    float lerp_w, b2, one_m_b2, eps, wd_factor, l2_wd, step_size, bc2_sqrt;
};

__device__ __forceinline__ float lerp_torch(float a, float b, float w) {
    // ATen lerp: weight < 0.5 ? a + w*(b-a) : b - (b-a)*(1-w)
    const float d = b - a;
    return w < 0.5f ? fmaf(w, d, a) : fmaf(-d, 1.f - w, b);
}

__device__ __forceinline__ void adam_elem(float& p, float& g, float& m, float& v, const AdamParams& ap) {
    if (ap.wd_factor != 1.f) p = p * ap.wd_factor;  // AdamW
    if (ap.l2_wd != 0.f) g = fmaf(ap.l2_wd, p, g);   // Adam
    m = lerp_torch(m, g, ap.lerp_w);
    v = fmaf(ap.one_m_b2 * g, g, v * ap.b2);
    const float denom = sqrtf(v) / ap.bc2_sqrt + ap.eps;
    p = fmaf(ap.step_size, m / denom, p);
}

}  // namespace ga
