// he_math.h -- device-side float32 vector / quaternion helpers (xyzw, Z-up) for gfx950 kernels.
// The quaternion formulas follow puffer_phc/torch_utils.py so the imitation kernel evaluates the
// same float32 expressions torch does (the imitation TU is compiled with -ffp-contract=off).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define HE_DEV __device__ __forceinline__
// The imitation helpers (*_ref, tan_norm, angle / exp maps, heading, the reset-time hash) follow the
// reference's float32 torch rounding: each body carries `#pragma clang fp contract(off)`, so no
// multiply-add is fused even when they are inlined into a TU compiled with contraction (the physics
// kernel's fused imitation epilogue).

struct f3 { float x, y, z; };
struct f4 { float x, y, z, w; };

HE_DEV f3 operator+(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
HE_DEV f3 operator-(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
HE_DEV f3 operator*(f3 a, float s) { return f3{a.x * s, a.y * s, a.z * s}; }
HE_DEV float dot3(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
HE_DEV f3 cross3(f3 a, f3 b) { return f3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
HE_DEV float norm3(f3 a) { return sqrtf(dot3(a, a)); }
HE_DEV f4 qconj(f4 q) { return f4{-q.x, -q.y, -q.z, q.w}; }
HE_DEV f4 qneg(f4 q) { return f4{-q.x, -q.y, -q.z, -q.w}; }

// torch_utils.py:54-75 (8-multiplication form)
HE_DEV f4 qmul_ref(f4 a, f4 b) {
#pragma clang fp contract(off)
    float x1 = a.x, y1 = a.y, z1 = a.z, w1 = a.w, x2 = b.x, y2 = b.y, z2 = b.z, w2 = b.w;
    float ww = (z1 + x1) * (x2 + y2);
    float yy = (w1 - y1) * (w2 + z2);
    float zz = (w1 + y1) * (w2 - z2);
    float xx = ww + yy + zz;
    float qq = 0.5f * (xx + (z1 - x1) * (x2 - y2));
    float w = qq - ww + (z1 - y1) * (y2 - z2);
    float x = qq - xx + (x1 + w1) * (x2 + w2);
    float y = qq - yy + (w1 - x1) * (y2 + z2);
    float z = qq - zz + (z1 + y1) * (w2 - x2);
    return f4{x, y, z, w};
}

// torch_utils.py:273-281 my_quat_rotate
HE_DEV f3 qrot_ref(f4 q, f3 v) {
#pragma clang fp contract(off)
    float s = 2.0f * (q.w * q.w) - 1.0f;
    // the cross product written out here (cross3 is a shared helper, compiled with contraction in
    // the physics TU)
    f3 c = f3{q.y * v.z - q.z * v.y, q.z * v.x - q.x * v.z, q.x * v.y - q.y * v.x};
    float d = v.x * q.x + v.y * q.y + v.z * q.z;
    return f3{v.x * s + c.x * q.w * 2.0f + q.x * d * 2.0f, v.y * s + c.y * q.w * 2.0f + q.y * d * 2.0f,
              v.z * s + c.z * q.w * 2.0f + q.z * d * 2.0f};
}

// torch_utils.py:284-297: (tan, norm) = (q*ex, q*ez)
HE_DEV void tan_norm(f4 q, float* o) {
#pragma clang fp contract(off)
    f3 t = qrot_ref(q, f3{1.f, 0.f, 0.f});
    f3 n = qrot_ref(q, f3{0.f, 0.f, 1.f});
    o[0] = t.x; o[1] = t.y; o[2] = t.z; o[3] = n.x; o[4] = n.y; o[5] = n.z;
}

HE_DEV float normalize_angle(float x) {
#pragma clang fp contract(off)
    return atan2f(sinf(x), cosf(x)); }

// torch_utils.py:85-106 -- angle; axis written when non-null
HE_DEV float q_angle_axis(f4 q, f3* axis) {
#pragma clang fp contract(off)
    float s = sqrtf(1.0f - q.w * q.w);
    float angle = normalize_angle(2.0f * acosf(q.w));
    bool mask = fabsf(s) > 1e-5f;  // NaN -> false
    if (axis) *axis = mask ? f3{q.x / s, q.y / s, q.z / s} : f3{0.f, 0.f, 1.f};
    return mask ? angle : 0.0f;
}

// torch_utils.py:143-150
HE_DEV f3 q_to_exp_map(f4 q) {
#pragma clang fp contract(off)
    f3 ax;
    float a = q_angle_axis(q, &ax);
    return ax * a;
}

// torch_utils.py:334-365 exp_map_to_quat = exp_map_to_angle_axis + quat_from_angle_axis
// (normalize and quat_unit clamp the norm at 1e-9), float32 in torch's operation order
HE_DEV f4 exp_map_to_quat_ref(f3 e) {
#pragma clang fp contract(off)
    float angle = sqrtf(e.x * e.x + e.y * e.y + e.z * e.z);
    f3 axis = f3{e.x / angle, e.y / angle, e.z / angle};
    angle = normalize_angle(angle);
    if (!(fabsf(angle) > 1e-5f)) { angle = 0.0f; axis = f3{0.f, 0.f, 1.f}; }
    float theta = angle / 2.0f;
    float n = fmaxf(sqrtf(axis.x * axis.x + axis.y * axis.y + axis.z * axis.z), 1e-9f);
    float st = sinf(theta);
    f4 q = f4{axis.x / n * st, axis.y / n * st, axis.z / n * st, cosf(theta)};
    float qn = fmaxf(sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w), 1e-9f);
    return f4{q.x / qn, q.y / qn, q.z / qn, q.w / qn};
}

// torch_utils.py:109-131 in torch's float32 operation order (sequential dot product)
HE_DEV f4 slerp_ref(f4 q0, f4 q1, float t) {
#pragma clang fp contract(off)
    float c = q0.x * q1.x;
    c = c + q0.y * q1.y;
    c = c + q0.z * q1.z;
    c = c + q0.w * q1.w;
    if (c < 0.0f) q1 = qneg(q1);
    c = fabsf(c);
    float half = acosf(c);
    float s = sqrtf(1.0f - c * c);
    float ra = sinf((1.0f - t) * half) / s, rb = sinf(t * half) / s;
    f4 o = f4{ra * q0.x + rb * q1.x, ra * q0.y + rb * q1.y, ra * q0.z + rb * q1.z, ra * q0.w + rb * q1.w};
    if (fabsf(s) < 0.001f) o = f4{0.5f * q0.x + 0.5f * q1.x, 0.5f * q0.y + 0.5f * q1.y, 0.5f * q0.z + 0.5f * q1.z,
                                  0.5f * q0.w + 0.5f * q1.w};
    if (c >= 1.0f) o = q0;
    return o;
}

// torch_utils.py:368-380: x-axis heading on the xy plane
HE_DEV float calc_heading(f4 q) {
#pragma clang fp contract(off)
    f3 d = qrot_ref(q, f3{1.f, 0.f, 0.f});
    return atan2f(d.y, d.x);
}
// torch_utils.py:353-358 quat_from_angle_axis(h, z) (normalize then quat_unit)
HE_DEV f4 heading_quat(float h) {
#pragma clang fp contract(off)
    float s = sinf(h / 2.0f), c = cosf(h / 2.0f);
    float n = fmaxf(sqrtf(s * s + c * c), 1e-9f);
    return f4{0.f, 0.f, s / n, c / n};
}

// ---- clean rotation helpers used by the physics kernel (not bit-matched to torch) --------
HE_DEV f4 qmul(f4 a, f4 b) {
    return f4{a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x,
              a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z};
}
HE_DEV f4 qnormalize(f4 q) {
    float n2 = q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w;
    if (n2 < 1e-24f) return f4{0.f, 0.f, 0.f, 1.f};
    float r = rsqrtf(n2);
    return f4{q.x * r, q.y * r, q.z * r, q.w * r};
}
// rotation matrix columns of q
HE_DEV void qcols(f4 q, f3& c0, f3& c1, f3& c2) {
    float x = q.x, y = q.y, z = q.z, w = q.w;
    c0 = f3{1 - 2 * (y * y + z * z), 2 * (x * y + z * w), 2 * (x * z - y * w)};
    c1 = f3{2 * (x * y - z * w), 1 - 2 * (x * x + z * z), 2 * (y * z + x * w)};
    c2 = f3{2 * (x * z + y * w), 2 * (y * z - x * w), 1 - 2 * (x * x + y * y)};
}
HE_DEV f3 qapply(f4 q, f3 v) {  // R(q) v
    f3 qv = f3{q.x, q.y, q.z};
    f3 t = cross3(qv, v) * 2.f;
    return v + t * q.w + cross3(qv, t);
}

// motion_lib.py:526-535 sample_time_interval, float32 ops as torch does them
HE_DEV float sample_time_interval(float phase, float len) {
#pragma clang fp contract(off)
    const float curr = (float)(1.0 / 30.0);
    float x = (phase * len) / curr;
    long long k = (long long)x;
    return (float)k * curr;
}

// counter-based uniform in [0,1) shared with the oracle (splitmix64 finaliser)
HE_DEV float hash_uniform(uint64_t seed, uint64_t step, uint32_t env) {
#pragma clang fp contract(off)
    uint64_t z = seed * 0x9E3779B97F4A7C15ull ^ (step + 0x632BE59BD9B4E019ull) * 0xBF58476D1CE4E5B9ull ^
                 ((uint64_t)env + 0x2545F4914F6CDD1Dull) * 0x94D049BB133111EBull;
    z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27; z *= 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (float)(z >> 40) * (1.0f / 16777216.0f);
}
