/*
 * ORACLE — test infrastructure only.  The rounding of the reference's BLAS-dispatched products.
 *
 * Julia hands every dense Float64 product the reference writes with `*` (other than a 2x2*2x2 or
 * 3x3*3x3 matrix product, which LinearAlgebra.matmul2x2!/3x3! evaluate without FMA) to its
 * OpenBLAS through BLAS.gemm! / gemv! / dot.  OpenBLAS's x86-64 kernels accumulate with FMA, so
 * those products do not round as a left fold of separately rounded terms.  This header restates,
 * per call shape the reference makes, the operation order of OpenBLAS 0.3.29 (SkylakeX kernels,
 * the build numpy ships here), pinned bit for bit against that library through its Fortran
 * interface (scipy_dgemm_64_ / scipy_dgemv_64_ / scipy_ddot_64_, the entry points Julia's
 * ccall binds) by tests/test_oracle_blas.py:
 *
 *   dgemm, any M x N, K <= 4 (the small-matrix kernel; also the Haswell/SkylakeX packed kernels):
 *        C[i,j] = fma(a_{K-1}, b_{K-1}, ... fma(a_1, b_1, a_0*b_0))      (accumulate k = 0, 1, ...)
 *   dgemv 'T', m = 2 rows (dgemv_t_4.c tail, contracted by the compiler):
 *        y[j] = fma(A[0,j], x_0, A[1,j]*x_1)
 *   dgemv 'N', m = 2 rows, n = 2 (dgemv_n_4.c tail loop):  y[i] = fma(A[i,1], x_1, A[i,0]*x_0)
 *   dgemv 'N', m = 2 rows, n = 4 (dgemv_n_4.c unrolled tail):
 *        y[i] = fma(A[i,0], x_0, A[i,1]*x_1) + fma(A[i,2], x_2, A[i,3]*x_3)
 *   ddot, n = 2:  fma(x_1, y_1, x_0*y_0)
 *
 * or_blas selects the convention for every such product in the oracle: 1 (the default) = as above,
 * 0 = the round-1..5 left fold of separately rounded products (kept for tools/blas_replay.py, which
 * counts the decisions the two conventions split).  Where it is used:
 *   CollisionDetection/src/utils.jl:24      GetRectanglePts  R*pts           dgemm 2x2 * 2x5
 *   CollisionDetection/src/utils.jl:48-49   SAT projections  transpose(M)*n  dgemv 'T' 2x5
 *   HybridAstar/src/hybrid_astar_utils.jl:109,123  cubic_fit pinv(A)*B (dgemv 'N' 2x2), Rmat*path (dgemm K=2)
 *   OptimalControl/ILQR/ILQR.jl:56-66       the Riccati products (dgemm, shapes in or_ilqr.c)
 *   OptimalControl/ILQR/ILQR.jl:76          Klist*(xtilde .- xn)              dgemv 'N' 2x4
 *   OptimalControl/MPPI/src/MPPIUtils.jl:45 λ * u' * inv(Σ) * d  = ((λu')*Σ⁻¹)*d: dgemv 'T' 2x2, ddot 2
 */
#ifndef OR_BLAS_H
#define OR_BLAS_H

extern int or_blas;

/* dgemm element with K = 2 */
static inline double blk2(double a0, double b0, double a1, double b1) {
  return or_blas ? __builtin_fma(a1, b1, a0 * b0) : a0 * b0 + a1 * b1;
}
/* dgemm element with K = 4 (operands a[k*sa], b[k*sb]) */
static inline double blk4(const double* a, int sa, const double* b, int sb) {
  double acc = a[0] * b[0];
  if (or_blas)
    for (int k = 1; k < 4; k++) acc = __builtin_fma(a[k * sa], b[k * sb], acc);
  else
    for (int k = 1; k < 4; k++) acc = acc + a[k * sa] * b[k * sb];
  return acc;
}
/* dgemv 'T' with two rows: column j of A (a0, a1) against x */
static inline double blv_t2(double a0, double x0, double a1, double x1) {
  return or_blas ? __builtin_fma(a0, x0, a1 * x1) : a0 * x0 + a1 * x1;
}
/* dgemv 'N', 2 x 2: row (a0, a1) against x */
static inline double blv_n22(double a0, double x0, double a1, double x1) {
  return or_blas ? __builtin_fma(a1, x1, a0 * x0) : a0 * x0 + a1 * x1;
}
/* dgemv 'N', 2 x 4: row a[0..3] (stride sa) against x[0..3] */
static inline double blv_n24(const double* a, int sa, const double* x) {
  if (or_blas)
    return __builtin_fma(a[0], x[0], a[sa] * x[1]) + __builtin_fma(a[2 * sa], x[2], a[3 * sa] * x[3]);
  double acc = a[0] * x[0];
  for (int c = 1; c < 4; c++) acc = acc + a[c * sa] * x[c];
  return acc;
}
/* ddot, n = 2 */
static inline double bl_dot2(double x0, double y0, double x1, double y1) {
  return or_blas ? __builtin_fma(x1, y1, x0 * y0) : x0 * y0 + x1 * y1;
}

#endif
