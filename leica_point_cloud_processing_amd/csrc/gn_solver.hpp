// gn_solver.hpp -- host Gauss-Newton solve of the GICP objective from its moments
// (MGICP_SOLVER_GN, the north star's "6x6 J'WJ / J'Wr" solve).
//
// Not a PCL 1.8.1 algorithm: PCL 1.8.1 only has the BFGS path (gicp.hpp
// estimateRigidTransformationBFGS, restated in pcl_bfgs.hpp).  For a fixed correspondence set the
// objective sum_i r_i' M_i r_i is an exact quadratic in A = [R | t] (DESIGN.md "The moment form"):
// with Y = A - T0 expressed about the centre c (Y[:,3] = dt + dR c) and G = B + Y Q,
//     f * m = S0 + sum_ai Y_ai (B_ai + G_ai)
// where S0, B (3x4) and Q (6x10 symmetric blocks) are the 74 moments of one device pass
// (gn_moments_kernel).  Poses are updated on the left about c:
//     p^ = R s + t - c,   T <- [Exp(w) | v] T,   J_i = [-[p^_i]x | I],
// so H = sum J'MJ and b = sum J'Mr at ANY pose are again linear in the moments: the whole inner
// solve runs on the host in microseconds, and a multi-GPU run needs one all-reduce of the moments
// per outer iteration.  Checker: oracle/gicp_ref.c estimate_gn (ref_params.solver = 1).
#pragma once
#include <cmath>
#include <cstring>

namespace mgicp {
namespace gn {

inline int sym_a(int a, int b) {
  static const int t[3][3] = {{0, 1, 2}, {1, 3, 4}, {2, 4, 5}};
  return t[a][b];
}
inline int sym_w(int i, int j) {
  static const int t[4][4] = {{0, 1, 2, 3}, {1, 4, 5, 6}, {2, 5, 7, 8}, {3, 6, 8, 9}};
  return t[i][j];
}

struct Pose {
  double R[3][3];
  double t[3];
};

struct Problem {
  const double* mom;  // kMomVals moments taken at T0
  double T0[3][4];    // correspondence transform (float entries widened)
  double c[3];        // expansion centre
  // Q entry for M block (a, b) and w pair (i, j)
  double q(int a, int b, int i, int j) const { return mom[13 + 10 * sym_a(a, b) + sym_w(i, j)]; }
};

// f * m at pose P; with H != nullptr also H = sum J'MJ and gv = sum J'Mr (half gradient)
inline double eval(const Problem& pb, const Pose& P, double H[6][6], double gv[6]) {
  const double* mo = pb.mom;
  double Y[3][4], E[3][4];  // Y = A - T0 about c; E = [R | R c + t - c] (p^ = E w)
  for (int a = 0; a < 3; ++a) {
    double u = P.t[a] - pb.T0[a][3];
    double e = P.t[a] - pb.c[a];
    for (int k = 0; k < 3; ++k) {
      Y[a][k] = P.R[a][k] - pb.T0[a][k];
      u += Y[a][k] * pb.c[k];
      E[a][k] = P.R[a][k];
      e += P.R[a][k] * pb.c[k];
    }
    Y[a][3] = u;
    E[a][3] = e;
  }
  double G[3][4];  // sum (M r)_b w_i
  for (int b = 0; b < 3; ++b)
    for (int i = 0; i < 4; ++i) {
      double acc = mo[1 + 4 * b + i];
      for (int cc = 0; cc < 3; ++cc)
        for (int j = 0; j < 4; ++j) acc += Y[cc][j] * pb.q(b, cc, i, j);
      G[b][i] = acc;
    }
  double fm = mo[0];
  for (int a = 0; a < 3; ++a)
    for (int i = 0; i < 4; ++i) fm += Y[a][i] * (mo[1 + 4 * a + i] + G[a][i]);
  if (!H) return fm;
  // Z[e][a] = sum p^_e (M r)_a,  N[e][a][b] = sum p^_e M_ab,  K[e][f][a][b] = sum p^_e p^_f M_ab
  double Z[3][3], N[3][3][3], K[3][3][3][3];
  for (int e = 0; e < 3; ++e)
    for (int a = 0; a < 3; ++a) {
      double z = 0.0;
      for (int i = 0; i < 4; ++i) z += E[e][i] * G[a][i];
      Z[e][a] = z;
    }
  for (int e = 0; e < 3; ++e)
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) {
        double s = 0.0;
        for (int i = 0; i < 4; ++i) s += E[e][i] * pb.q(a, b, i, 3);
        N[e][a][b] = s;
      }
  for (int e = 0; e < 3; ++e)
    for (int f = 0; f < 3; ++f)
      for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) {
          double s = 0.0;
          for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) s += E[e][i] * E[f][j] * pb.q(a, b, i, j);
          K[e][f][a][b] = s;
        }
  static const int eps[3][3][3] = {{{0, 0, 0}, {0, 0, 1}, {0, -1, 0}},
                                   {{0, 0, -1}, {0, 0, 0}, {1, 0, 0}},
                                   {{0, 1, 0}, {-1, 0, 0}, {0, 0, 0}}};
  // rotation block: J_w' M r = p^ x (M r), J_w' M J_v = [p^]x M, J_w' M J_w = -[p^]x M [p^]x
  for (int i = 0; i < 3; ++i) {
    double s = 0.0;
    for (int j = 0; j < 3; ++j)
      for (int k = 0; k < 3; ++k) s += eps[i][j][k] * Z[j][k];
    gv[i] = s;
    gv[3 + i] = G[i][3];
  }
  for (int i = 0; i < 3; ++i)
    for (int l = 0; l < 3; ++l) {
      double wv = 0.0, ww = 0.0;
      for (int j = 0; j < 3; ++j)
        for (int k = 0; k < 3; ++k) {
          if (!eps[i][j][k]) continue;
          wv += eps[i][j][k] * N[j][k][l];
          for (int mm = 0; mm < 3; ++mm)
            for (int n = 0; n < 3; ++n)
              if (eps[mm][n][l]) ww -= eps[i][j][k] * eps[mm][n][l] * K[j][n][k][mm];
        }
      H[i][3 + l] = wv;
      H[3 + l][i] = wv;
      H[i][l] = ww;
      H[3 + i][3 + l] = pb.q(i, l, 3, 3);
    }
  return fm;
}

// Cholesky solve of H x = -b; false when H is not positive definite
inline bool chol_solve(const double H[6][6], const double b[6], double x[6]) {
  double L[6][6];
  std::memset(L, 0, sizeof(L));
  for (int j = 0; j < 6; ++j) {
    double d = H[j][j];
    for (int k = 0; k < j; ++k) d -= L[j][k] * L[j][k];
    if (!(d > 0.0)) return false;
    L[j][j] = std::sqrt(d);
    for (int i = j + 1; i < 6; ++i) {
      double s = H[i][j];
      for (int k = 0; k < j; ++k) s -= L[i][k] * L[j][k];
      L[i][j] = s / L[j][j];
    }
  }
  double y[6];
  for (int i = 0; i < 6; ++i) {
    double s = -b[i];
    for (int k = 0; k < i; ++k) s -= L[i][k] * y[k];
    y[i] = s / L[i][i];
  }
  for (int i = 5; i >= 0; --i) {
    double s = y[i];
    for (int k = i + 1; k < 6; ++k) s -= L[k][i] * x[k];
    x[i] = s / L[i][i];
  }
  return true;
}

// Rodrigues: Exp of a rotation vector
inline void so3_exp(const double w[3], double Rx[3][3]) {
  const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  const double th = std::sqrt(th2);
  double a, b;
  if (th < 1e-8) {
    a = 1.0 - th2 / 6.0;
    b = 0.5 - th2 / 24.0;
  } else {
    double sth, cth;
    ::sincos(th, &sth, &cth);  // glibc sincos, as the gcc-built oracle restatement calls it (r06)
    a = sth / th;
    b = (1.0 - cth) / th2;
  }
  const double W[3][3] = {{0, -w[2], w[1]}, {w[2], 0, -w[0]}, {-w[1], w[0], 0}};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      const double w2 = W[i][0] * W[0][j] + W[i][1] * W[1][j] + W[i][2] * W[2][j];
      Rx[i][j] = (i == j ? 1.0 : 0.0) + a * W[i][j] + b * w2;
    }
}

// P' = [Exp(s w) | s v] applied on the left about c
inline Pose retract(const Pose& P, const double c[3], const double xi[6], double s) {
  const double w[3] = {s * xi[0], s * xi[1], s * xi[2]};
  double Rx[3][3];
  so3_exp(w, Rx);
  Pose Q;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j)
      Q.R[i][j] = Rx[i][0] * P.R[0][j] + Rx[i][1] * P.R[1][j] + Rx[i][2] * P.R[2][j];
    Q.t[i] = Rx[i][0] * (P.t[0] - c[0]) + Rx[i][1] * (P.t[1] - c[1]) +
             Rx[i][2] * (P.t[2] - c[2]) + c[i] + s * xi[3 + i];
  }
  return Q;
}

// Damped (step-halving) Gauss-Newton from pose P on the moments of pb; at most max_iter solves.
// Returns false when the normal matrix is singular (PCL would have thrown from its solver).
inline bool solve(const Problem& pb, Pose& P, int max_iter, int* n_evals) {
  double H[6][6], gv[6];
  double fm = eval(pb, P, H, gv);
  ++*n_evals;
  for (int it = 0; it < max_iter; ++it) {
    double xi[6];
    if (!chol_solve(H, gv, xi)) return false;
    Pose Q = P;
    double s = 1.0;
    bool ok = false;
    for (int h = 0; h < 8; ++h, s *= 0.5) {
      Q = retract(P, pb.c, xi, s);
      if (eval(pb, Q, nullptr, nullptr) <= fm) {
        ok = true;
        break;
      }
    }
    if (!ok) break;  // no descent along the GN direction: at the minimum to rounding
    P = Q;
    double step = 0.0;
    for (int k = 0; k < 6; ++k) step = std::fmax(step, std::fabs(s * xi[k]));
    if (step < 1e-12) break;
    fm = eval(pb, P, H, gv);
    ++*n_evals;
  }
  return true;
}

}  // namespace gn
}  // namespace mgicp
