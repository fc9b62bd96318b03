// rmsf_device.h -- device math shared by the HIP translation units
// (rmsf_kernels.hip: the two-pass superpose/accumulate kernels; fused.hip:
// the single-read fused sweep): the f32-faithful transform of RMSF.py:99-101
// / 133-135 and the QCP solve of qcprot (RMSF.py:43-51).  Both kernels call
// exactly this code, so a frame's rotation and its transformed coordinates
// come out of the same instruction sequence on either path.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

// ---------------------------------------------------------------------------
// f32-faithful superposition transform of RMSF.py:99-101 / 133-135.
//   p = f32(f64(p) - com); p = f32(f64(p) @ R); p = f32(f64(p) + ref_com)
__device__ __forceinline__ void apply_xform(float &x, float &y, float &z, const double *__restrict__ t,
                                            double rc0, double rc1, double rc2) {
  const float p0 = (float)((double)x - t[9]);
  const float p1 = (float)((double)y - t[10]);
  const float p2 = (float)((double)z - t[11]);
  const double d0 = p0, d1 = p1, d2 = p2;
  // out_b = sum_a p_a R[a][b]   (np.dot(positions, R), R row-major), as the
  // host BLAS dgemm accumulates it: an FMA chain over a = 0, 1, 2 from
  // p_0 R[0][b] (tests/test_rotation_rounding.py: numpy's dot equals this
  // chain bit for bit, the unfused sum in only 60-75 % of values).  Explicit fma,
  // so the rounding order does not depend on -ffp-contract.
  const float r0 = (float)__builtin_fma(d2, t[6], __builtin_fma(d1, t[3], d0 * t[0]));
  const float r1 = (float)__builtin_fma(d2, t[7], __builtin_fma(d1, t[4], d0 * t[1]));
  const float r2 = (float)__builtin_fma(d2, t[8], __builtin_fma(d1, t[5], d0 * t[2]));
  x = (float)((double)r0 + rc0);
  y = (float)((double)r1 + rc1);
  z = (float)((double)r2 + rc2);
}

// ---------------------------------------------------------------------------
// QCP: the published quaternion-characteristic-polynomial algorithm
// (D. Theobald, Acta Cryst A 61:478, 2005; P. Liu et al., J Comput Chem
// 31:1561, 2010), as used by MDAnalysis.lib.qcprot (RMSF.py:48).  A is the
// row-major inner product sum_i mob_i[a] ref_i[b]; rot is applied as x @ rot.
// SURVEY.md Appendix A.2-A.3 gives the exact sequence followed here.
__host__ __device__ inline void qcp_solve(const double *A, double E0, double len, double *rot,
                                          double *rmsd) {
  const double Sxx = A[0], Sxy = A[1], Sxz = A[2];
  const double Syx = A[3], Syy = A[4], Syz = A[5];
  const double Szx = A[6], Szy = A[7], Szz = A[8];

  const double Sxx2 = Sxx * Sxx, Syy2 = Syy * Syy, Szz2 = Szz * Szz;
  const double Sxy2 = Sxy * Sxy, Syz2 = Syz * Syz, Sxz2 = Sxz * Sxz;
  const double Syx2 = Syx * Syx, Szy2 = Szy * Szy, Szx2 = Szx * Szx;

  const double SyzSzymSyySzz2 = 2.0 * (Syz * Szy - Syy * Szz);
  const double Sxx2Syy2Szz2Syz2Szy2 = Syy2 + Szz2 - Sxx2 + Syz2 + Szy2;

  const double C2 = -2.0 * (Sxx2 + Syy2 + Szz2 + Sxy2 + Syx2 + Sxz2 + Szx2 + Syz2 + Szy2);
  const double C1 = 8.0 * (Sxx * Syz * Szy + Syy * Szx * Sxz + Szz * Sxy * Syx - Sxx * Syy * Szz -
                           Syz * Szx * Sxy - Szy * Syx * Sxz);

  const double SxzpSzx = Sxz + Szx, SyzpSzy = Syz + Szy, SxypSyx = Sxy + Syx;
  const double SyzmSzy = Syz - Szy, SxzmSzx = Sxz - Szx, SxymSyx = Sxy - Syx;
  const double SxxpSyy = Sxx + Syy, SxxmSyy = Sxx - Syy;
  const double Sxy2Sxz2Syx2Szx2 = Sxy2 + Sxz2 - Syx2 - Szx2;

  const double C0 =
      Sxy2Sxz2Syx2Szx2 * Sxy2Sxz2Syx2Szx2 +
      (Sxx2Syy2Szz2Syz2Szy2 + SyzSzymSyySzz2) * (Sxx2Syy2Szz2Syz2Szy2 - SyzSzymSyySzz2) +
      (-(SxzpSzx) * (SyzmSzy) + (SxymSyx) * (SxxmSyy - Szz)) *
          (-(SxzmSzx) * (SyzpSzy) + (SxymSyx) * (SxxmSyy + Szz)) +
      (-(SxzpSzx) * (SyzpSzy) - (SxypSyx) * (SxxpSyy - Szz)) *
          (-(SxzmSzx) * (SyzmSzy) - (SxypSyx) * (SxxpSyy + Szz)) +
      (+(SxypSyx) * (SyzpSzy) + (SxzpSzx) * (SxxmSyy + Szz)) *
          (-(SxymSyx) * (SyzmSzy) + (SxzpSzx) * (SxxpSyy + Szz)) +
      (+(SxypSyx) * (SyzmSzy) + (SxzmSzx) * (SxxmSyy - Szz)) *
          (-(SxymSyx) * (SyzpSzy) + (SxzmSzx) * (SxxpSyy - Szz));

  // Newton-Raphson on the quartic, from lambda = E0 (upper bound).
  double l = E0;
  for (int i = 0; i < 50; ++i) {
    const double old = l;
    const double x2 = l * l;
    const double b = (x2 + C2) * l;
    const double a = b + C1;
    const double delta = (a * l + C0) / (2.0 * x2 * l + b + a);
    l -= delta;
    if (fabs(l - old) < fabs(1e-11 * l)) break;
  }
  *rmsd = sqrt(fabs(2.0 * (E0 - l) / len));

  const double a11 = SxxpSyy + Szz - l, a12 = SyzmSzy, a13 = -SxzmSzx, a14 = SxymSyx;
  const double a21 = SyzmSzy, a22 = SxxmSyy - Szz - l, a23 = SxypSyx, a24 = SxzpSzx;
  const double a31 = a13, a32 = a23, a33 = Syy - Sxx - Szz - l, a34 = SyzpSzy;
  const double a41 = a14, a42 = a24, a43 = a34, a44 = Szz - SxxpSyy - l;
  const double a3344_4334 = a33 * a44 - a43 * a34, a3244_4234 = a32 * a44 - a42 * a34;
  const double a3243_4233 = a32 * a43 - a42 * a33, a3143_4133 = a31 * a43 - a41 * a33;
  const double a3144_4134 = a31 * a44 - a41 * a34, a3142_4132 = a31 * a42 - a41 * a32;
  double q1 = a22 * a3344_4334 - a23 * a3244_4234 + a24 * a3243_4233;
  double q2 = -a21 * a3344_4334 + a23 * a3144_4134 - a24 * a3143_4133;
  double q3 = a21 * a3244_4234 - a22 * a3144_4134 + a24 * a3142_4132;
  double q4 = -a21 * a3243_4233 + a22 * a3143_4133 - a23 * a3142_4132;
  double qsqr = q1 * q1 + q2 * q2 + q3 * q3 + q4 * q4;

  const double evecprec = 1e-6;
  if (qsqr < evecprec) {
    q1 = a12 * a3344_4334 - a13 * a3244_4234 + a14 * a3243_4233;
    q2 = -a11 * a3344_4334 + a13 * a3144_4134 - a14 * a3143_4133;
    q3 = a11 * a3244_4234 - a12 * a3144_4134 + a14 * a3142_4132;
    q4 = -a11 * a3243_4233 + a12 * a3143_4133 - a13 * a3142_4132;
    qsqr = q1 * q1 + q2 * q2 + q3 * q3 + q4 * q4;
    if (qsqr < evecprec) {
      const double a1324_1423 = a13 * a24 - a14 * a23, a1224_1422 = a12 * a24 - a14 * a22;
      const double a1223_1322 = a12 * a23 - a13 * a22, a1124_1421 = a11 * a24 - a14 * a21;
      const double a1123_1321 = a11 * a23 - a13 * a21, a1122_1221 = a11 * a22 - a12 * a21;
      q1 = a42 * a1324_1423 - a43 * a1224_1422 + a44 * a1223_1322;
      q2 = -a41 * a1324_1423 + a43 * a1124_1421 - a44 * a1123_1321;
      q3 = a41 * a1224_1422 - a42 * a1124_1421 + a44 * a1122_1221;
      q4 = -a41 * a1223_1322 + a42 * a1123_1321 - a43 * a1122_1221;
      qsqr = q1 * q1 + q2 * q2 + q3 * q3 + q4 * q4;
      if (qsqr < evecprec) {
        q1 = a32 * a1324_1423 - a33 * a1224_1422 + a34 * a1223_1322;
        q2 = -a31 * a1324_1423 + a33 * a1124_1421 - a34 * a1123_1321;
        q3 = a31 * a1224_1422 - a32 * a1124_1421 + a34 * a1122_1221;
        q4 = -a31 * a1223_1322 + a32 * a1123_1321 - a33 * a1122_1221;
        qsqr = q1 * q1 + q2 * q2 + q3 * q3 + q4 * q4;
        if (qsqr < evecprec) {
          rot[0] = rot[4] = rot[8] = 1.0;
          rot[1] = rot[2] = rot[3] = rot[5] = rot[6] = rot[7] = 0.0;
          return;
        }
      }
    }
  }
  const double normq = sqrt(qsqr);
  q1 /= normq;
  q2 /= normq;
  q3 /= normq;
  q4 /= normq;
  const double a2 = q1 * q1, x2 = q2 * q2, y2 = q3 * q3, z2 = q4 * q4;
  const double xy = q2 * q3, az = q1 * q4, zx = q4 * q2, ay = q1 * q3, yz = q3 * q4, ax = q1 * q2;
  rot[0] = a2 + x2 - y2 - z2;
  rot[1] = 2 * (xy + az);
  rot[2] = 2 * (zx - ay);
  rot[3] = 2 * (xy - az);
  rot[4] = a2 - x2 + y2 - z2;
  rot[5] = 2 * (yz + ax);
  rot[6] = 2 * (zx + ay);
  rot[7] = 2 * (yz - ax);
  rot[8] = a2 - x2 - y2 + z2;
}

