/* ORACLE — test infrastructure only (see oracle/__init__.py).
 *
 * Plain-C restatement of the SpMV the reference executes: mvmult(A,x) = A*x
 * (IterativeLinearSolver.py:94-106) dispatches to scipy sparsetools'
 * csr_matvec (scipy 1.15.3, sparsetools/csr.h), whose published algorithm is
 *
 *     for i in rows:  sum = y[i] (= 0, result is np.zeros);
 *                     for jj in [Ap[i], Ap[i+1]): sum += Ax[jj] * Xx[Aj[jj]];
 *
 * i.e. a sequential per-row sum in STORED order, product rounded before the
 * add (scipy's x86-64 baseline build has no FMA).  Compiled with
 * -ffp-contract=off so the C compiler cannot fuse the multiply-add either.
 * tests/test_oracle_golden.py checks this bit-for-bit against scipy and the
 * committed golden vectors.
 *
 * Also: csr_diagonal (scipy csr_diagonal: sum of the entries with col==row,
 * in stored order, starting from 0) used by the Jacobi preconditioner.
 */
#include <stdint.h>

void oracle_csr_matvec(int64_t n, const int32_t *Ap, const int32_t *Aj,
                       const double *Ax, const double *x, double *y)
{
    for (int64_t i = 0; i < n; ++i) {
        double sum = 0.0;
        for (int64_t jj = Ap[i]; jj < Ap[i + 1]; ++jj) {
            double prod = Ax[jj] * x[Aj[jj]];
            sum = sum + prod;
        }
        y[i] = sum;
    }
}

void oracle_csr_diagonal(int64_t n, const int32_t *Ap, const int32_t *Aj,
                         const double *Ax, double *d)
{
    for (int64_t i = 0; i < n; ++i) {
        double s = 0.0;
        for (int64_t jj = Ap[i]; jj < Ap[i + 1]; ++jj)
            if (Aj[jj] == i) s = s + Ax[jj];
        d[i] = s;
    }
}
