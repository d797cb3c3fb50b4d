// vmas_dual.hpp -- forward-mode dual numbers for the gradient path (csrc/vmas_grad.hip).
//
// A Dual carries an fp32 value -- computed with exactly the forward step's fp32 operations, so
// the value part of a dual step equals the forward step -- and K tangents, the derivatives of
// that value with respect to K chosen inputs.  Comparisons look at the value only, so branches,
// clamps and first-minimum selections take the forward's path and the derivative is that of the
// taken branch (what torch.autograd gives the reference's tensor program).  Derivatives at the
// kinks follow torch's conventions where the reference meets them: sqrt'(0) := 0 (the norm of a
// zero vector, torch.linalg.vector_norm's backward), |x|'(0) = sign(0) = 0.
#pragma once

#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#include <math.h>
#endif

#define VDD __host__ __device__ __forceinline__

namespace vmas_dual {

constexpr int kTangents = 8;  // inputs per pass: a step's Jacobian takes ceil(n_in / 8) passes

struct Dual {
    float v;
    float d[kTangents];
    VDD Dual() : v(0.f) {
#pragma unroll
        for (int k = 0; k < kTangents; ++k) d[k] = 0.f;
    }
    VDD Dual(float x) : v(x) {  // a constant (zero tangents)
#pragma unroll
        for (int k = 0; k < kTangents; ++k) d[k] = 0.f;
    }
};

// x with tangent 1 in slot k (k < 0 or k >= kTangents: a constant)
VDD Dual seed(float x, int k) {
    Dual r(x);
    if (k >= 0 && k < kTangents) r.d[k] = 1.f;
    return r;
}

VDD Dual operator+(const Dual& a, const Dual& b) {
    Dual r;
    r.v = a.v + b.v;
#pragma unroll
    for (int k = 0; k < kTangents; ++k) r.d[k] = a.d[k] + b.d[k];
    return r;
}
VDD Dual operator-(const Dual& a, const Dual& b) {
    Dual r;
    r.v = a.v - b.v;
#pragma unroll
    for (int k = 0; k < kTangents; ++k) r.d[k] = a.d[k] - b.d[k];
    return r;
}
VDD Dual operator-(const Dual& a) {
    Dual r;
    r.v = -a.v;
#pragma unroll
    for (int k = 0; k < kTangents; ++k) r.d[k] = -a.d[k];
    return r;
}
VDD Dual operator*(const Dual& a, const Dual& b) {
    Dual r;
    r.v = a.v * b.v;
#pragma unroll
    for (int k = 0; k < kTangents; ++k) r.d[k] = a.d[k] * b.v + a.v * b.d[k];
    return r;
}
VDD Dual operator/(const Dual& a, const Dual& b) {
    Dual r;
    r.v = a.v / b.v;
#pragma unroll
    for (int k = 0; k < kTangents; ++k) r.d[k] = (a.d[k] - r.v * b.d[k]) / b.v;
    return r;
}
// mixed operands: the float is a constant
VDD Dual operator+(const Dual& a, float b) { return a + Dual(b); }
VDD Dual operator+(float a, const Dual& b) { return Dual(a) + b; }
VDD Dual operator-(const Dual& a, float b) { return a - Dual(b); }
VDD Dual operator-(float a, const Dual& b) { return Dual(a) - b; }
VDD Dual operator*(const Dual& a, float b) {
    Dual r;
    r.v = a.v * b;
#pragma unroll
    for (int k = 0; k < kTangents; ++k) r.d[k] = a.d[k] * b;
    return r;
}
VDD Dual operator*(float a, const Dual& b) {
    Dual r;
    r.v = a * b.v;
#pragma unroll
    for (int k = 0; k < kTangents; ++k) r.d[k] = a * b.d[k];
    return r;
}
VDD Dual operator/(const Dual& a, float b) {
    Dual r;
    r.v = a.v / b;
#pragma unroll
    for (int k = 0; k < kTangents; ++k) r.d[k] = a.d[k] / b;
    return r;
}
VDD Dual operator/(float a, const Dual& b) { return Dual(a) / b; }

#define VMAS_DUAL_CMP(op)                                                       \
    VDD bool operator op(const Dual& a, const Dual& b) { return a.v op b.v; }   \
    VDD bool operator op(const Dual& a, float b) { return a.v op b; }           \
    VDD bool operator op(float a, const Dual& b) { return a op b.v; }
VMAS_DUAL_CMP(<)
VMAS_DUAL_CMP(>)
VMAS_DUAL_CMP(<=)
VMAS_DUAL_CMP(>=)
VMAS_DUAL_CMP(==)
VMAS_DUAL_CMP(!=)
#undef VMAS_DUAL_CMP

VDD Dual chain(const Dual& a, float value, float slope) {
    Dual r;
    r.v = value;
#pragma unroll
    for (int k = 0; k < kTangents; ++k) r.d[k] = slope * a.d[k];
    return r;
}

VDD Dual sqrtf(const Dual& a) {
    const float s = ::sqrtf(a.v);
    return chain(a, s, s > 0.f ? 0.5f / s : 0.f);
}
VDD Dual expf(const Dual& a) {
    const float e = ::expf(a.v);
    return chain(a, e, e);
}
VDD Dual log1pf(const Dual& a) { return chain(a, ::log1pf(a.v), 1.f / (1.f + a.v)); }
VDD Dual cosf(const Dual& a) { return chain(a, ::cosf(a.v), -::sinf(a.v)); }
VDD Dual sinf(const Dual& a) { return chain(a, ::sinf(a.v), ::cosf(a.v)); }
VDD Dual fabsf(const Dual& a) { return chain(a, ::fabsf(a.v), a.v > 0.f ? 1.f : (a.v < 0.f ? -1.f : 0.f)); }

}  // namespace vmas_dual
