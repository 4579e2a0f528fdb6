// ba_device.h — device-side math shared by the libmiba HIP kernels.
//
// Per-observation residual + analytic local Jacobian (the replacement of the
// reference's two AutoDiff cost functors, Jet<double,14> x 2 per observation):
//   ReprojectionConstraint::operator()  /root/reference/src/OptimizationUtils.cpp:25-49
//   DepthPrior::operator()              /root/reference/src/OptimizationUtils.cpp:72-94
// robustified with Ceres HuberLoss(HUB_P_*) + Corrector (rho'' <= 0 => sqrt(rho')
// scaling), see OptimizationUtils.cpp:223-226, BundleAdjustmentConfig.h:47-50.
// The pose Jacobian is taken w.r.t. the Sophus right perturbation T*exp(delta),
// delta = [upsilon, omega] (local_parameterization_se3.hpp:17-37), which equals
// Ceres' ambient Jacobian x Dx_this_mul_exp_x_at_0 (se3.hpp:113-182).
#pragma once
#include <hip/hip_runtime.h>
#include <float.h>

namespace miba {

struct BaConsts {
    double sw_r, sw_d, sw_k;   // sqrt(1/N), sqrt(WEIGHT_UNPR/N), sqrt(WEIGHT_INTRINSICS)
    double a_r, b_r, a_d, b_d; // Huber a and b = a^2 (reprojection, depth)
    double min_diag, max_diag; // LM diagonal clamp
};

// Eigen toRotationMatrix of q = (w=p[3], x=p[0], y=p[1], z=p[2])  (OptimizationUtils.cpp:36-41)
__device__ __forceinline__ void quat_R(const double* __restrict__ p, double R[9]) {
    const double x = p[0], y = p[1], z = p[2], w = p[3];
    const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w;
    const double txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

// 1/x: v_rcp_f64 + two Newton steps (within an ulp or two of the IEEE quotient; five dependent
// ops instead of the ~10-instruction f64 division sequence on the per-observation critical path)
__device__ __forceinline__ double rcp_f64(double x) {
    double y = __builtin_amdgcn_rcp(x);
    double e = __builtin_fma(-x, y, 1.0);
    y = __builtin_fma(y, e, y);
    e = __builtin_fma(-x, y, 1.0);
    return __builtin_fma(y, e, y);
}

// Huber rho(s) and sqrt(rho'(s))  (Ceres HuberLoss::Evaluate; Corrector)
__device__ __forceinline__ void huber(double s, double a, double b, double& rho0, double& sq_rho1) {
    if (s > b) {
        const double r = sqrt(s);
        rho0 = 2.0 * a * r - b;
        sq_rho1 = sqrt(fmax(DBL_MIN, a * rcp_f64(r)));
    } else {
        rho0 = s;
        sq_rho1 = 1.0;
    }
}

struct ObsEval {
    double f[3];   // robustified residual (reproj u, v, depth)
    double cost;   // 0.5 rho_r + 0.5 rho_d
    bool ok;
};

// Residual only (candidate evaluation).
__device__ __forceinline__ void eval_obs(const BaConsts& c, const double* __restrict__ pose,
                                         const double* __restrict__ X, const double* __restrict__ K,
                                         double uo, double vo, double depth, ObsEval& o) {
    double R[9];
    quat_R(pose, R);
    const double d0 = X[0] - pose[4], d1 = X[1] - pose[5], d2 = X[2] - pose[6];
    const double x = R[0] * d0 + R[3] * d1 + R[6] * d2;
    const double y = R[1] * d0 + R[4] * d1 + R[7] * d2;
    const double z = R[2] * d0 + R[5] * d1 + R[8] * d2;
    const double iz = rcp_f64(z);
    const double u = (K[0] * x + K[2] * z) * iz;
    const double v = (K[1] * y + K[3] * z) * iz;
    const double r0 = c.sw_r * (u - uo), r1 = c.sw_r * (v - vo), r2 = c.sw_d * (depth - z);
    double rr, gr, rd, gd;
    huber(r0 * r0 + r1 * r1, c.a_r, c.b_r, rr, gr);
    huber(r2 * r2, c.a_d, c.b_d, rd, gd);
    o.cost = 0.5 * rr + 0.5 * rd;
    o.f[0] = gr * r0; o.f[1] = gr * r1; o.f[2] = gd * r2;
    o.ok = isfinite(o.cost) && isfinite(u) && isfinite(v);
}

// Residual + robustified local Jacobians.
//   jc[r*6+d] (d: upsilon xyz, omega xyz), jp[r*3+i], jk[r*4+i] (rows 0,1; depth row has none)
__device__ __forceinline__ void lin_obs(const BaConsts& c, const double* __restrict__ pose,
                                        const double* __restrict__ X, const double* __restrict__ K,
                                        double uo, double vo, double depth, ObsEval& o, double jc[18],
                                        double jp[9], double jk[8]) {
    double R[9];
    quat_R(pose, R);
    const double d0 = X[0] - pose[4], d1 = X[1] - pose[5], d2 = X[2] - pose[6];
    const double x = R[0] * d0 + R[3] * d1 + R[6] * d2;
    const double y = R[1] * d0 + R[4] * d1 + R[7] * d2;
    const double z = R[2] * d0 + R[5] * d1 + R[8] * d2;
    const double fx = K[0], fy = K[1], cx = K[2], cy = K[3];
    const double iz = rcp_f64(z);
    const double u = (fx * x + cx * z) * iz;
    const double v = (fy * y + cy * z) * iz;
    const double r0 = c.sw_r * (u - uo), r1 = c.sw_r * (v - vo), r2 = c.sw_d * (depth - z);
    double rr, gr, rd, gd;
    huber(r0 * r0 + r1 * r1, c.a_r, c.b_r, rr, gr);
    huber(r2 * r2, c.a_d, c.b_d, rd, gd);
    o.cost = 0.5 * rr + 0.5 * rd;
    o.f[0] = gr * r0; o.f[1] = gr * r1; o.f[2] = gd * r2;
    o.ok = isfinite(o.cost) && isfinite(u) && isfinite(v);
    const double su = gr * c.sw_r;
    const double a00 = su * fx * iz, a02 = -su * fx * x * iz * iz;
    const double a11 = su * fy * iz, a12 = -su * fy * y * iz * iz;
    const double dz = -gd * c.sw_d;
    // row 0: [a00, 0, a02] ; row 1: [0, a11, a12] ; row 2: [0, 0, dz]
    // d pC / d upsilon = -I ; d pC / d omega = [pC]x = [[0,-z,y],[z,0,-x],[-y,x,0]]
    // translation columns: -A ; omega columns: A . P
    jc[0] = -a00; jc[1] = 0.0; jc[2] = -a02;
    jc[3] = -a02 * y; jc[4] = a02 * x - a00 * z; jc[5] = a00 * y;
    jc[6] = 0.0; jc[7] = -a11; jc[8] = -a12;
    jc[9] = a11 * z - a12 * y; jc[10] = a12 * x; jc[11] = -a11 * x;
    jc[12] = 0.0; jc[13] = 0.0; jc[14] = -dz;
    jc[15] = -dz * y; jc[16] = dz * x; jc[17] = 0.0;
    // d pC / d X = R^T : (R^T)_{k i} = R[i*3+k]
    jp[0] = a00 * R[0] + a02 * R[2];
    jp[1] = a00 * R[3] + a02 * R[5];
    jp[2] = a00 * R[6] + a02 * R[8];
    jp[3] = a11 * R[1] + a12 * R[2];
    jp[4] = a11 * R[4] + a12 * R[5];
    jp[5] = a11 * R[7] + a12 * R[8];
    jp[6] = dz * R[2];
    jp[7] = dz * R[5];
    jp[8] = dz * R[8];
    jk[0] = su * x * iz; jk[1] = 0.0; jk[2] = su; jk[3] = 0.0;
    jk[4] = 0.0; jk[5] = su * y * iz; jk[6] = 0.0; jk[7] = su;
}

// Structural zeros of the local Jacobian (lin_obs): jc row 0 has no upsilon_y entry, row 1 no
// upsilon_x, row 2 only upsilon_z / omega_x / omega_y; jk rows are [fx-col, 0, 1-col, 0] and
// [0, fy-col, 0, 1-col] (times su). The camera-side sums therefore have 9 entries that are zero for
// every observation — U(0,1), C(0,1), C(0,3), C(1,0), C(1,2), Ukk(0,1), Ukk(0,3), Ukk(1,2), Ukk(2,3) —
// and the rest need 80 products instead of 160. CAM_NZ packed sums per observation:
//   [0, 20)  U upper-packed without U(0,1)      [20, 40) C without its 4 zeros
//   [40, 46) g = Jc^T f                          [46, 52) Ukk nonzeros (00, 02, 11, 13, 22, 33)
//   [52, 56) gk = Jk^T f                         [56]     cost
static constexpr int CAM_NZ = 57;
// The packed sums in two halves (for callers short of registers): CAM_NZ_U = U (20) | g (6) | cost -> packed
// [0, 20), [40, 46), 56; CAM_NZ_C = C (20) | Ukk (6) | gk (4) -> packed [20, 40), [46, 56).
static constexpr int CAM_NZ_U = 27, CAM_NZ_C = 30;
__device__ __forceinline__ int cam_nz_u_index(int i) { return i < 20 ? i : (i < 26 ? 40 + (i - 20) : 56); }
__device__ __forceinline__ int cam_nz_c_index(int i) { return i < 20 ? 20 + i : 46 + (i - 20); }
__device__ __forceinline__ void cam_accum_u(double* a, const double jc[18], const double f[3], double cost, bool cam) {
    const double c0 = jc[0], c2 = jc[2], c3 = jc[3], c4 = jc[4], c5 = jc[5];
    const double e1 = jc[7], e2 = jc[8], e3 = jc[9], e4 = jc[10], e5 = jc[11];
    const double h2 = jc[14], h3 = jc[15], h4 = jc[16];
    if (cam) {
        a[0] += c0 * c0; a[1] += c0 * c2; a[2] += c0 * c3; a[3] += c0 * c4; a[4] += c0 * c5;
        a[5] += e1 * e1; a[6] += e1 * e2; a[7] += e1 * e3; a[8] += e1 * e4; a[9] += e1 * e5;
        a[10] += c2 * c2 + e2 * e2 + h2 * h2;
        a[11] += c2 * c3 + e2 * e3 + h2 * h3;
        a[12] += c2 * c4 + e2 * e4 + h2 * h4;
        a[13] += c2 * c5 + e2 * e5;
        a[14] += c3 * c3 + e3 * e3 + h3 * h3;
        a[15] += c3 * c4 + e3 * e4 + h3 * h4;
        a[16] += c3 * c5 + e3 * e5;
        a[17] += c4 * c4 + e4 * e4 + h4 * h4;
        a[18] += c4 * c5 + e4 * e5;
        a[19] += c5 * c5 + e5 * e5;
        a[20] += c0 * f[0];
        a[21] += e1 * f[1];
        a[22] += c2 * f[0] + e2 * f[1] + h2 * f[2];
        a[23] += c3 * f[0] + e3 * f[1] + h3 * f[2];
        a[24] += c4 * f[0] + e4 * f[1] + h4 * f[2];
        a[25] += c5 * f[0] + e5 * f[1];
    }
    a[26] += cost;
}
__device__ __forceinline__ void cam_accum_c(double* a, const double jc[18], const double jk[8], const double f[3],
                                            bool cam) {
    const double c0 = jc[0], c2 = jc[2], c3 = jc[3], c4 = jc[4], c5 = jc[5];
    const double e1 = jc[7], e2 = jc[8], e3 = jc[9], e4 = jc[10], e5 = jc[11];
    const double k0 = jk[0], su = jk[2], k1 = jk[5];
    if (cam) {
        // C[i][m]: row 0 pairs with jk columns 0, 2; row 1 with 1, 3
        a[0] += c0 * k0; a[1] += c0 * su;                        // C00, C02
        a[2] += e1 * k1; a[3] += e1 * su;                        // C11, C13
        a[4] += c2 * k0; a[5] += e2 * k1; a[6] += c2 * su; a[7] += e2 * su;      // C2*
        a[8] += c3 * k0; a[9] += e3 * k1; a[10] += c3 * su; a[11] += e3 * su;    // C3*
        a[12] += c4 * k0; a[13] += e4 * k1; a[14] += c4 * su; a[15] += e4 * su;  // C4*
        a[16] += c5 * k0; a[17] += e5 * k1; a[18] += c5 * su; a[19] += e5 * su;  // C5*
    }
    a[20] += k0 * k0; a[21] += k0 * su; a[22] += k1 * k1; a[23] += k1 * su; a[24] += su * su; a[25] += su * su;
    a[26] += k0 * f[0]; a[27] += k1 * f[1]; a[28] += su * f[0]; a[29] += su * f[1];
}
__device__ __forceinline__ void cam_accum(double* a, const double jc[18], const double jk[8],
                                          const double f[3], double cost, bool cam) {
    double u[CAM_NZ_U], cc[CAM_NZ_C];
#pragma unroll
    for (int i = 0; i < CAM_NZ_U; ++i) u[i] = a[cam_nz_u_index(i)];
#pragma unroll
    for (int i = 0; i < CAM_NZ_C; ++i) cc[i] = a[cam_nz_c_index(i)];
    cam_accum_u(u, jc, f, cost, cam);
    cam_accum_c(cc, jc, jk, f, cam);
#pragma unroll
    for (int i = 0; i < CAM_NZ_U; ++i) a[cam_nz_u_index(i)] = u[i];
#pragma unroll
    for (int i = 0; i < CAM_NZ_C; ++i) a[cam_nz_c_index(i)] = cc[i];
}
// Expand the packed sums into the CAMDATA (U 21 | C 24 | g 6) and SEGINTR (Ukk 10 | gk 4 | cost)
// layouts: element e of [camdata | segintr] (66 values) from the packed array p.
__device__ __forceinline__ double cam_unpack(const double* p, int e) {
    // U upper-packed (i <= j): q = 6 i - i (i - 1) / 2 + (j - i); q = 1 is U(0,1) == 0
    if (e < 21) return e == 0 ? p[0] : (e == 1 ? 0.0 : p[e - 1]);
    if (e < 45) {  // C[i][m], e - 21 = 4 i + m
        const int i = (e - 21) >> 2, m = (e - 21) & 3;
        if (i == 0) return m == 0 ? p[20] : (m == 2 ? p[21] : 0.0);
        if (i == 1) return m == 1 ? p[22] : (m == 3 ? p[23] : 0.0);
        return p[24 + 4 * (i - 2) + m];
    }
    if (e < 51) return p[40 + (e - 45)];
    if (e < 61) {  // Ukk packed (m <= l): 00 01 02 03 11 12 13 22 23 33
        switch (e - 51) {
            case 0: return p[46];
            case 2: return p[47];
            case 4: return p[48];
            case 6: return p[49];
            case 7: return p[50];
            case 9: return p[51];
            default: return 0.0;
        }
    }
    return p[52 + (e - 61)];  // gk (4), cost
}

// Sophus T * exp(delta)  (se3.hpp:725-746, so3.hpp:537-571, so3.hpp:339-356)
__device__ __forceinline__ void se3_plus(const double* __restrict__ T, const double* __restrict__ d,
                                         double* __restrict__ out) {
    const double ox = d[3], oy = d[4], oz = d[5];
    const double theta_sq = ox * ox + oy * oy + oz * oz;
    double imag, real;
    double V[9];
    if (theta_sq < 1e-20) {  // theta < 1e-10: Sophus' small-angle branch (V = the rotation itself)
        const double t4 = theta_sq * theta_sq;
        imag = 0.5 - (1.0 / 48.0) * theta_sq + (1.0 / 3840.0) * t4;
        real = 1.0 - (1.0 / 8.0) * theta_sq + (1.0 / 384.0) * t4;
        const double qd0[4] = {imag * ox, imag * oy, imag * oz, real};
        quat_R(qd0, V);
    } else {
        double a, b;
        if (theta_sq < 1.0) {
            // theta < 1 (every LM step short of a 1 rad rotation): sin(theta / 2) = h ps(h^2), cos(theta / 2) =
            // pc(h^2), (theta - sin theta) / theta^3 = pb(theta^2) by their Taylor series (truncated below 3e-17) in
            // FMA form: imag = sin(h) / theta = ps / 2, a = 2 sin^2(h) / theta^2 = ps^2 / 2 — no square root,
            // division or library sincos on the camera step's critical path
            const double h2 = 0.25 * theta_sq;
            double ps = 1.0 / 6227020800.0;  // 1/13!
            ps = __builtin_fma(ps, -h2, 1.0 / 39916800.0);
            ps = __builtin_fma(ps, -h2, 1.0 / 362880.0);
            ps = __builtin_fma(ps, -h2, 1.0 / 5040.0);
            ps = __builtin_fma(ps, -h2, 1.0 / 120.0);
            ps = __builtin_fma(ps, -h2, 1.0 / 6.0);
            ps = __builtin_fma(ps, -h2, 1.0);
            double pc = 1.0 / 87178291200.0;  // 1/14!
            pc = __builtin_fma(pc, -h2, 1.0 / 479001600.0);
            pc = __builtin_fma(pc, -h2, 1.0 / 3628800.0);
            pc = __builtin_fma(pc, -h2, 1.0 / 40320.0);
            pc = __builtin_fma(pc, -h2, 1.0 / 720.0);
            pc = __builtin_fma(pc, -h2, 1.0 / 24.0);
            pc = __builtin_fma(pc, -h2, 0.5);
            real = __builtin_fma(pc, -h2, 1.0);
            imag = 0.5 * ps;
            a = 0.5 * ps * ps;
            double pb = 1.0 / 355687428096000.0;  // 1/17!
            pb = __builtin_fma(pb, -theta_sq, 1.0 / 1307674368000.0);
            pb = __builtin_fma(pb, -theta_sq, 1.0 / 6227020800.0);
            pb = __builtin_fma(pb, -theta_sq, 1.0 / 39916800.0);
            pb = __builtin_fma(pb, -theta_sq, 1.0 / 362880.0);
            pb = __builtin_fma(pb, -theta_sq, 1.0 / 5040.0);
            pb = __builtin_fma(pb, -theta_sq, 1.0 / 120.0);
            b = __builtin_fma(pb, -theta_sq, 1.0 / 6.0);
        } else {
            const double theta = sqrt(theta_sq);
            double sh, ch;
            sincos(0.5 * theta, &sh, &ch);
            imag = sh / theta;
            real = ch;
            // sin(theta) and 1 - cos(theta) from the half-angle pair (2 sin^2(theta / 2) avoids the cancellation)
            a = (2.0 * sh * sh) / theta_sq;
            b = (theta - 2.0 * sh * ch) / (theta_sq * theta);
        }
        const double Om[9] = {0, -oz, oy, oz, 0, -ox, -oy, ox, 0};
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const double o2 = Om[i * 3 + 0] * Om[0 * 3 + j] + Om[i * 3 + 1] * Om[1 * 3 + j] + Om[i * 3 + 2] * Om[2 * 3 + j];
                V[i * 3 + j] = (i == j ? 1.0 : 0.0) + a * Om[i * 3 + j] + b * o2;
            }
    }
    const double qd[4] = {imag * ox, imag * oy, imag * oz, real};
    double td[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) td[i] = V[i * 3 + 0] * d[0] + V[i * 3 + 1] * d[1] + V[i * 3 + 2] * d[2];
    const double qx = T[0], qy = T[1], qz = T[2], qw = T[3];
    const double uv0 = 2 * (qy * td[2] - qz * td[1]);
    const double uv1 = 2 * (qz * td[0] - qx * td[2]);
    const double uv2 = 2 * (qx * td[1] - qy * td[0]);
    out[4] = T[4] + (td[0] + qw * uv0 + (qy * uv2 - qz * uv1));
    out[5] = T[5] + (td[1] + qw * uv1 + (qz * uv0 - qx * uv2));
    out[6] = T[6] + (td[2] + qw * uv2 + (qx * uv1 - qy * uv0));
    const double bx = qd[0], by = qd[1], bz = qd[2], bw = qd[3];
    double nw = qw * bw - qx * bx - qy * by - qz * bz;
    double nx = qw * bx + qx * bw + qy * bz - qz * by;
    double ny = qw * by + qy * bw + qz * bx - qx * bz;
    double nz = qw * bz + qz * bw + qx * by - qy * bx;
    const double sq = nx * nx + ny * ny + nz * nz + nw * nw;
    if (sq != 1.0) {
        // 2 / (1 + sq) = 1 / (1 + e / 2), e = sq - 1: 1 - e / 2 + e^2 / 4 is exact to double for |e| < 1e-6 (a unit
        // quaternion times a unit quaternion: e is a few ulp), a division otherwise
        const double e = sq - 1.0;
        const double f = fabs(e) < 1e-6 ? __builtin_fma(e, __builtin_fma(e, 0.25, -0.5), 1.0) : 2.0 / (1.0 + sq);
        nx *= f; ny *= f; nz *= f; nw *= f;
    }
    out[0] = nx; out[1] = ny; out[2] = nz; out[3] = nw;
}

}  // namespace miba
