// Device-side activation functions by ActCode (ddl_ops.h), shared by the standalone activation
// kernels (kernels/layer_ops.hip) and the generic recurrent cells (kernels/rnn.hip).
// act_d takes the forward OUTPUT y (GELU: its input x), so backward passes need no pre-activation.
#pragma once
#include "ddl_common.h"
#include "ddl_ops.h"

namespace ddl {

constexpr float kSeluAlpha = 1.6732632423543772f, kSeluScale = 1.0507009873554805f;

__device__ __forceinline__ float act_f(int code, float x) {
  switch (code) {
    case ACT_C_RELU: return fmaxf(x, 0.f);
    case ACT_C_TANH: return tanhf(x);
    case ACT_C_SIGMOID: return 1.f / (1.f + __expf(-x));
    case ACT_C_HARD_SIGMOID: return fminf(fmaxf(0.2f * x + 0.5f, 0.f), 1.f);
    case ACT_C_ELU: return x > 0.f ? x : expm1f(x);
    case ACT_C_SELU: return kSeluScale * (x > 0.f ? x : kSeluAlpha * expm1f(x));
    case ACT_C_SOFTPLUS: return x > 20.f ? x : log1pf(__expf(x));
    case ACT_C_GELU: return gelu_f(x);
    default: return x;
  }
}

__device__ __forceinline__ float act_d(int code, float v) {
  switch (code) {
    case ACT_C_RELU: return v > 0.f ? 1.f : 0.f;
    case ACT_C_TANH: return 1.f - v * v;
    case ACT_C_SIGMOID: return v * (1.f - v);
    case ACT_C_HARD_SIGMOID: return (v > 0.f && v < 1.f) ? 0.2f : 0.f;
    case ACT_C_ELU: return v > 0.f ? 1.f : v + 1.f;
    case ACT_C_SELU: return v > 0.f ? kSeluScale : v + kSeluScale * kSeluAlpha;
    case ACT_C_SOFTPLUS: return -expm1f(-v);
    case ACT_C_GELU: return gelu_grad_f(v);
    default: return 1.f;
  }
}

}  // namespace ddl
