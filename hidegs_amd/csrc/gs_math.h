// gs_math.h -- device math for the gfx950 Gaussian splatting rasterizer.
//
// Written from the published method, not from any existing implementation:
//   * 3D Gaussian Splatting (Kerbl et al., SIGGRAPH 2023): anisotropic Gaussians
//     with covariance Sigma = R S S^T R^T, projected with the local affine (EWA)
//     approximation Sigma' = J W Sigma W^T J^T (Zwicker et al., "EWA Splatting",
//     2002), front-to-back alpha compositing over 16x16 screen tiles.
//   * Real spherical harmonics up to degree 3 for view-dependent colour.
//   * A screen-space low-pass filter of variance s = 0.1 px^2 added to Sigma'
//     with the energy-preserving opacity factor sqrt(det Sigma' / det(Sigma'+sI))
//     (the "2D Mip filter" of Mip-Splatting, Yu et al., CVPR 2024).
//
// Symmetric matrices are stored as their unique entries:
//   3x3: {xx, xy, xz, yy, yz, zz};  2x2: {a = xx, b = xy, c = yy}.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gsm {

constexpr float kLowPass = 0.1f;       // screen-space filter variance (px^2)
constexpr float kNear = 0.2f;          // near-plane distance (camera units)
constexpr float kFrustumGuard = 1.3f;  // clamp of x/z, y/z to 1.3 * tan(fov/2)
constexpr float kAlphaMax = 0.99f;
constexpr float kAlphaMin = 1.0f / 255.0f;
constexpr float kTransmittanceMin = 0.0001f;

struct f3 {
    float x, y, z;
};
__device__ __forceinline__ f3 mk3(float x, float y, float z) { return f3{x, y, z}; }

struct sym3 {
    float xx, xy, xz, yy, yz, zz;
};
struct sym2 {
    float a, b, c;
};

// Camera matrices arrive as 16 floats laid out for row vectors (p' = [p,1] * M),
// i.e. column j of the math matrix is M[4*0+j], M[4*1+j], ... .
struct Cam {
    float v[16];  // world -> view
    float p[16];  // world -> clip
};
__device__ __forceinline__ f3 to_view(const float* m, f3 q)
{
    return mk3(m[0] * q.x + m[4] * q.y + m[8] * q.z + m[12], m[1] * q.x + m[5] * q.y + m[9] * q.z + m[13],
               m[2] * q.x + m[6] * q.y + m[10] * q.z + m[14]);
}
__device__ __forceinline__ float4 to_clip(const float* m, f3 q)
{
    return make_float4(m[0] * q.x + m[4] * q.y + m[8] * q.z + m[12], m[1] * q.x + m[5] * q.y + m[9] * q.z + m[13],
                       m[2] * q.x + m[6] * q.y + m[10] * q.z + m[14], m[3] * q.x + m[7] * q.y + m[11] * q.z + m[15]);
}

// Rotation matrix rows of quaternion (w, x, y, z) taken as given.
struct Rot {
    float r[3][3];  // r[i][j] = R_ij
};
__device__ __forceinline__ Rot quat_rot(float w, float x, float y, float z)
{
    Rot R;
    R.r[0][0] = 1.f - 2.f * (y * y + z * z);
    R.r[0][1] = 2.f * (x * y - w * z);
    R.r[0][2] = 2.f * (x * z + w * y);
    R.r[1][0] = 2.f * (x * y + w * z);
    R.r[1][1] = 1.f - 2.f * (x * x + z * z);
    R.r[1][2] = 2.f * (y * z - w * x);
    R.r[2][0] = 2.f * (x * z - w * y);
    R.r[2][1] = 2.f * (y * z + w * x);
    R.r[2][2] = 1.f - 2.f * (x * x + y * y);
    return R;
}

// Sigma = M^T M with M = S R^T... written directly: Sigma_ij = sum_k R_ik s_k^2 R_jk.
__device__ __forceinline__ sym3 covariance(f3 s, const Rot& R)
{
    float s0 = s.x * s.x, s1 = s.y * s.y, s2 = s.z * s.z;
    sym3 S;
    S.xx = R.r[0][0] * R.r[0][0] * s0 + R.r[0][1] * R.r[0][1] * s1 + R.r[0][2] * R.r[0][2] * s2;
    S.xy = R.r[0][0] * R.r[1][0] * s0 + R.r[0][1] * R.r[1][1] * s1 + R.r[0][2] * R.r[1][2] * s2;
    S.xz = R.r[0][0] * R.r[2][0] * s0 + R.r[0][1] * R.r[2][1] * s1 + R.r[0][2] * R.r[2][2] * s2;
    S.yy = R.r[1][0] * R.r[1][0] * s0 + R.r[1][1] * R.r[1][1] * s1 + R.r[1][2] * R.r[1][2] * s2;
    S.yz = R.r[1][0] * R.r[2][0] * s0 + R.r[1][1] * R.r[2][1] * s1 + R.r[1][2] * R.r[2][2] * s2;
    S.zz = R.r[2][0] * R.r[2][0] * s0 + R.r[2][1] * R.r[2][1] * s1 + R.r[2][2] * R.r[2][2] * s2;
    return S;
}

// Screen-space projection.  A = J W is the 2x3 Jacobian of pixel coordinates
// w.r.t. world position (rows a0, a1); Sigma' = A Sigma A^T.
struct Proj2 {
    float a0[3], a1[3];  // rows of A
    float tx, ty, tz;    // view-space mean (tx, ty clamped)
    bool clamp_x, clamp_y;
};
__device__ __forceinline__ Proj2 jacobian(const float* v, f3 mean, float fx, float fy, float tanx, float tany)
{
    Proj2 P;
    f3 t = to_view(v, mean);
    float limx = kFrustumGuard * tanx, limy = kFrustumGuard * tany;
    float ux = t.x / t.z, uy = t.y / t.z;
    P.clamp_x = ux < -limx || ux > limx;
    P.clamp_y = uy < -limy || uy > limy;
    ux = fminf(limx, fmaxf(-limx, ux));
    uy = fminf(limy, fmaxf(-limy, uy));
    P.tx = ux * t.z;
    P.ty = uy * t.z;
    P.tz = t.z;
    // J rows: [fx/z, 0, -fx x/z^2], [0, fy/z, -fy y/z^2]; W rows are view-matrix columns.
    float j00 = fx / t.z, j02 = -(fx * P.tx) / (t.z * t.z);
    float j11 = fy / t.z, j12 = -(fy * P.ty) / (t.z * t.z);
    for (int k = 0; k < 3; k++) {
        // W_{r,k} = v[4*k + r] for r = 0..2
        P.a0[k] = j00 * v[4 * k + 0] + j02 * v[4 * k + 2];
        P.a1[k] = j11 * v[4 * k + 1] + j12 * v[4 * k + 2];
    }
    return P;
}
__device__ __forceinline__ float quad(const float* u, const sym3& S, const float* w)
{
    // u^T S w
    float sw0 = S.xx * w[0] + S.xy * w[1] + S.xz * w[2];
    float sw1 = S.xy * w[0] + S.yy * w[1] + S.yz * w[2];
    float sw2 = S.xz * w[0] + S.yz * w[1] + S.zz * w[2];
    return u[0] * sw0 + u[1] * sw1 + u[2] * sw2;
}
__device__ __forceinline__ sym2 project(const Proj2& P, const sym3& S)
{
    return sym2{quad(P.a0, S, P.a0), quad(P.a0, S, P.a1), quad(P.a1, S, P.a1)};
}

// Real SH basis (degree <= 3) evaluated at unit direction d, 16 values.
__device__ __forceinline__ void sh_basis(int deg, f3 d, float* Y)
{
    const float C0 = 0.28209479177387814f, C1 = 0.4886025119029199f;
    float x = d.x, y = d.y, z = d.z;
    Y[0] = C0;
    if (deg < 1) return;
    Y[1] = -C1 * y;
    Y[2] = C1 * z;
    Y[3] = -C1 * x;
    if (deg < 2) return;
    float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    Y[4] = 1.0925484305920792f * xy;
    Y[5] = -1.0925484305920792f * yz;
    Y[6] = 0.31539156525252005f * (2.f * zz - xx - yy);
    Y[7] = -1.0925484305920792f * xz;
    Y[8] = 0.5462742152960396f * (xx - yy);
    if (deg < 3) return;
    Y[9] = -0.5900435899266435f * y * (3.f * xx - yy);
    Y[10] = 2.890611442640554f * xy * z;
    Y[11] = -0.4570457994644658f * y * (4.f * zz - xx - yy);
    Y[12] = 0.3731763325901154f * z * (2.f * zz - 3.f * xx - 3.f * yy);
    Y[13] = -0.4570457994644658f * x * (4.f * zz - xx - yy);
    Y[14] = 1.445305721320277f * z * (xx - yy);
    Y[15] = -0.5900435899266435f * x * (xx - 3.f * yy);
}
// Gradient of sum_k Y_k(d) * g_k w.r.t. d (g = per-basis weights), degree <= 3.
__device__ __forceinline__ f3 sh_basis_grad(int deg, f3 d, const float* g)
{
    const float C1 = 0.4886025119029199f;
    float x = d.x, y = d.y, z = d.z;
    float gx = 0.f, gy = 0.f, gz = 0.f;
    if (deg < 1) return mk3(0, 0, 0);
    gx += -C1 * g[3];
    gy += -C1 * g[1];
    gz += C1 * g[2];
    if (deg >= 2) {
        const float a = 1.0925484305920792f, b = 0.31539156525252005f, c = 0.5462742152960396f;
        gx += a * y * g[4] - a * z * g[7] + b * (-2.f * x) * g[6] + c * (2.f * x) * g[8];
        gy += a * x * g[4] - a * z * g[5] + b * (-2.f * y) * g[6] + c * (-2.f * y) * g[8];
        gz += -a * y * g[5] - a * x * g[7] + b * (4.f * z) * g[6];
    }
    if (deg >= 3) {
        const float k9 = -0.5900435899266435f, k10 = 2.890611442640554f, k11 = -0.4570457994644658f;
        const float k12 = 0.3731763325901154f, k13 = -0.4570457994644658f, k14 = 1.445305721320277f;
        const float k15 = -0.5900435899266435f;
        float xx = x * x, yy = y * y, zz = z * z;
        // d/dx
        gx += k9 * (6.f * x * y) * g[9] + k10 * (y * z) * g[10] + k11 * (-2.f * x * y) * g[11] +
              k12 * (-6.f * x * z) * g[12] + k13 * (4.f * zz - 3.f * xx - yy) * g[13] + k14 * (2.f * x * z) * g[14] +
              k15 * (3.f * xx - 3.f * yy) * g[15];
        // d/dy
        gy += k9 * (3.f * xx - 3.f * yy) * g[9] + k10 * (x * z) * g[10] + k11 * (4.f * zz - xx - 3.f * yy) * g[11] +
              k12 * (-6.f * y * z) * g[12] + k13 * (-2.f * x * y) * g[13] + k14 * (-2.f * y * z) * g[14] +
              k15 * (-6.f * x * y) * g[15];
        // d/dz
        gz += k10 * (x * y) * g[10] + k11 * (8.f * y * z) * g[11] + k12 * (6.f * zz - 3.f * xx - 3.f * yy) * g[12] +
              k13 * (8.f * x * z) * g[13] + k14 * (xx - yy) * g[14];
    }
    return mk3(gx, gy, gz);
}

// exp for the blend loops: one v_exp_f32 on x*log2(e).
__device__ __forceinline__ float fast_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }

}  // namespace gsm
