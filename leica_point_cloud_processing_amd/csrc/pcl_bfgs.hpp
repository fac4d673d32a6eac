// pcl_bfgs.hpp -- host-side 6-DoF solver of the engine, PCL 1.8.1 trajectory semantics.
//
// Restates pcl/registration/bfgs.h (a port of GSL's vector_bfgs2 with Fletcher's line
// search) and GICP::estimateRigidTransformationBFGS (registration/impl/gicp.hpp) so that
// the engine follows the same iterate sequence as the reference's PCL CPU GICP
// (SURVEY.md 8a a6, Appendix A.5).  Every objective evaluation is a device pass; the
// functor always returns f AND the gradient, and memoises the last state so the
// f / df / fdf cache protocol of bfgs.h costs no extra passes and yields identical values.
//
// Two details of PCL 1.8.1's interpolate() are kept exactly as published:
//   the cubic branch is guarded by !(fpb != fpa) (GSL: fpb is real), and the quadratic
//   minimum is accepted when curvature c > a (GSL: c > 0).
#pragma once
#include <cfloat>
#include <cmath>
#include <cstring>
#include <limits>

namespace mgicp {

struct Vec6 {
  double v[6];
  double& operator[](int i) { return v[i]; }
  double operator[](int i) const { return v[i]; }
};

inline double dot(const Vec6& a, const Vec6& b) {
  double r = 0;
  for (int i = 0; i < 6; ++i) r += a[i] * b[i];
  return r;
}
inline double norm(const Vec6& a) { return std::sqrt(dot(a, a)); }

enum BfgsStatus { kNegEps = -3, kNotStarted = -2, kRunning = -1, kSuccess = 0, kNoProgress = 1 };

// Functor concept: int eval(const Vec6& x, double& f, Vec6& g)  (0 = ok)
template <class Functor>
class PclBfgs {
 public:
  explicit PclBfgs(Functor& fn) : fn_(fn) {}

  double rho = 0.01, sigma = 0.01, tau1 = 9, tau2 = 0.05, tau3 = 0.5, step_size = 1;
  int order = 3, bracket_iters = 100, section_iters = 100;
  double f = 0;
  Vec6 gradient{};
  int error = 0;  // first functor error, aborts the solve

  int init(Vec6& x) {
    delta_f_ = 0;
    dx_ = Vec6{};
    call(x, f, gradient);
    x0_ = x;
    g0_ = gradient;
    g0norm_ = norm(g0_);
    for (int i = 0; i < 6; ++i) p_[i] = gradient[i] * -1 / g0norm_;
    pnorm_ = norm(p_);
    fp0_ = -g0norm_;
    x_alpha_ = x0_;
    x_key_ = 0;
    f_alpha_ = f;
    f_key_ = 0;
    g_alpha_ = g0_;
    g_key_ = 0;
    df_alpha_ = slope();
    df_key_ = 0;
    return kNotStarted;
  }

  int step(Vec6& x) {
    double alpha = 0.0, alpha1;
    const double f0 = f;
    if (pnorm_ == 0.0 || g0norm_ == 0.0 || fp0_ == 0) {
      dx_ = Vec6{};
      return kNoProgress;
    }
    if (delta_f_ < 0) {
      const double del = std::max(-delta_f_, 10 * std::numeric_limits<double>::epsilon() * std::fabs(f0));
      alpha1 = std::min(1.0, 2.0 * del / (-fp0_));
    } else {
      alpha1 = std::fabs(step_size);
    }
    const int status = line_search(alpha1, alpha);
    if (status != kSuccess || error) return error ? kNoProgress : status;
    {  // updatePosition
      double fa, dfa;
      apply_fdf(alpha, fa, dfa);
      f = f_alpha_;
      x = x_alpha_;
      gradient = g_alpha_;
    }
    delta_f_ = f - f0;
    {  // BFGS direction update
      Vec6 dx0, dg0;
      for (int i = 0; i < 6; ++i) {
        dx0[i] = x[i] - x0_[i];
        dg0[i] = gradient[i] - g0_[i];
      }
      dx_ = dx0;
      const double dxg = dot(dx0, gradient), dgg = dot(dg0, gradient), dxdg = dot(dx0, dg0);
      const double dgnorm = norm(dg0);
      double A, B;
      if (dxdg != 0) {
        B = dxg / dxdg;
        A = -(1.0 + dgnorm * dgnorm / dxdg) * B + dgg / dxdg;
      } else {
        B = 0;
        A = 0;
      }
      for (int i = 0; i < 6; ++i) {
        p_[i] = -A * dx0[i];
        p_[i] += -B * dg0[i];
        p_[i] += gradient[i];
      }
    }
    g0_ = gradient;
    x0_ = x;
    g0norm_ = norm(g0_);
    pnorm_ = norm(p_);
    const double dir = (dot(p_, gradient) > 0) ? -1.0 : 1.0;
    for (int i = 0; i < 6; ++i) p_[i] *= dir / pnorm_;
    pnorm_ = norm(p_);
    fp0_ = dot(p_, g0_);
    // changeDirection
    x_alpha_ = x0_;
    x_key_ = 0.0;
    f_key_ = 0.0;
    g_alpha_ = g0_;
    g_key_ = 0.0;
    df_alpha_ = slope();
    df_key_ = 0.0;
    return kSuccess;
  }

  int test_gradient(double eps) const {
    if (eps < 0) return kNegEps;
    return norm(gradient) < eps ? kSuccess : kRunning;
  }

 private:
  Functor& fn_;
  double delta_f_ = 0, fp0_ = 0, pnorm_ = 0, g0norm_ = 0;
  Vec6 x0_{}, g0_{}, dx_{}, p_{};
  double f_alpha_ = 0, df_alpha_ = 0;
  Vec6 x_alpha_{}, g_alpha_{};
  double f_key_ = 0, df_key_ = 0, x_key_ = 0, g_key_ = 0;

  void call(const Vec6& x, double& fv, Vec6& gv) {
    if (error) return;
    error = fn_.eval(x, fv, gv);
  }
  double slope() const { return dot(g_alpha_, p_); }
  void move_to(double alpha) {
    for (int i = 0; i < 6; ++i) x_alpha_[i] = x0_[i] + alpha * p_[i];
    x_key_ = alpha;
  }
  double apply_f(double alpha) {
    if (alpha == f_key_) return f_alpha_;
    move_to(alpha);
    Vec6 gtmp;
    call(x_alpha_, f_alpha_, gtmp);  // gradient computed too but not cached (bfgs.h applyF)
    f_key_ = alpha;
    return f_alpha_;
  }
  double apply_df(double alpha) {
    if (alpha == df_key_) return df_alpha_;
    move_to(alpha);
    if (alpha != g_key_) {
      double ftmp;
      call(x_alpha_, ftmp, g_alpha_);
      g_key_ = alpha;
    }
    df_alpha_ = slope();
    df_key_ = alpha;
    return df_alpha_;
  }
  void apply_fdf(double alpha, double& fv, double& dfv) {
    if (alpha == f_key_ && alpha == df_key_) {
      fv = f_alpha_;
      dfv = df_alpha_;
      return;
    }
    if (alpha == f_key_ || alpha == df_key_) {
      fv = apply_f(alpha);
      dfv = apply_df(alpha);
      return;
    }
    move_to(alpha);
    call(x_alpha_, f_alpha_, g_alpha_);
    f_key_ = alpha;
    g_key_ = alpha;
    df_alpha_ = slope();
    df_key_ = alpha;
    fv = f_alpha_;
    dfv = df_alpha_;
  }

  static double poly_eval(const double c[4], double x) {
    double v = c[3];
    v = v * x + c[2];
    v = v * x + c[1];
    v = v * x + c[0];
    return v;
  }
  static void check_extremum(const double c[4], double x, double& xmin, double& fmin) {
    const double y = poly_eval(c, x);
    if (y < fmin) {
      xmin = x;
      fmin = y;
    }
  }

  static double interpolate(double a, double fa, double fpa, double b, double fb, double fpb,
                            double xmin, double xmax, int ord) {
    double y, fmin;
    double ymin = (xmin - a) / (b - a);
    double ymax = (xmax - a) / (b - a);
    if (ymin > ymax) std::swap(ymin, ymax);
    if (ord > 2 && !(fpb != fpa) && fpb != std::numeric_limits<double>::infinity()) {
      fpa = fpa * (b - a);
      fpb = fpb * (b - a);
      const double eta = 3 * (fb - fa) - 2 * fpa - fpb;
      const double xi = fpa + fpb - 2 * (fb - fa);
      const double c[4] = {fa, fpa, eta, xi};
      y = ymin;
      fmin = poly_eval(c, ymin);
      check_extremum(c, ymax, y, fmin);
      const double qa = 3 * xi, qb = 2 * eta, qc = fpa;  // derivative c1 + 2c2 y + 3c3 y^2
      if (qa != 0.0) {
        const double disc = qb * qb - 4 * qa * qc;
        if (disc >= 0.0) {
          const double sq = std::sqrt(disc);
          double y0 = (-qb - sq) / (2 * qa), y1 = (-qb + sq) / (2 * qa);
          if (y0 > y1) std::swap(y0, y1);
          if (y0 > ymin && y0 < ymax) check_extremum(c, y0, y, fmin);
          if (y1 > ymin && y1 < ymax) check_extremum(c, y1, y, fmin);
        }
      } else if (qb != 0.0) {
        const double y0 = -qc / qb;
        if (y0 > ymin && y0 < ymax) check_extremum(c, y0, y, fmin);
      }
    } else {
      fpa = fpa * (b - a);
      const double fl = fa + ymin * (fpa + ymin * (fb - fa - fpa));
      const double fh = fa + ymax * (fpa + ymax * (fb - fa - fpa));
      const double c = 2 * (fb - fa - fpa);
      y = ymin;
      fmin = fl;
      if (fh < fmin) {
        y = ymax;
        fmin = fh;
      }
      if (c > a) {
        const double z = -fpa / c;
        if (z > ymin && z < ymax) {
          const double fz = fa + z * (fpa + z * (fb - fa - fpa));
          if (fz < fmin) {
            y = z;
            fmin = fz;
          }
        }
      }
    }
    return a + y * (b - a);
  }

  int line_search(double alpha1, double& alpha_new) {
    double f0, fp0, falpha, falpha_prev, fpalpha, fpalpha_prev, delta, alpha_next;
    double alpha = alpha1, alpha_prev = 0.0;
    double a, b, fa, fb, fpa, fpb;
    int i = 0;
    apply_fdf(0.0, f0, fp0);
    falpha_prev = f0;
    fpalpha_prev = fp0;
    a = 0.0;
    b = alpha;
    fa = f0;
    fb = 0.0;
    fpa = fp0;
    fpb = 0.0;
    const double nan = std::numeric_limits<double>::quiet_NaN();
    while (i++ < bracket_iters) {
      falpha = apply_f(alpha);
      if (falpha > f0 + alpha * rho * fp0 || falpha >= falpha_prev) {
        a = alpha_prev; fa = falpha_prev; fpa = fpalpha_prev;
        b = alpha; fb = falpha; fpb = nan;
        break;
      }
      fpalpha = apply_df(alpha);
      if (std::fabs(fpalpha) <= -sigma * fp0) {
        alpha_new = alpha;
        return kSuccess;
      }
      if (fpalpha >= 0) {
        a = alpha; fa = falpha; fpa = fpalpha;
        b = alpha_prev; fb = falpha_prev; fpb = fpalpha_prev;
        break;
      }
      delta = alpha - alpha_prev;
      {
        const double lower = alpha + delta;
        const double upper = alpha + tau1 * delta;
        alpha_next = interpolate(alpha_prev, falpha_prev, fpalpha_prev, alpha, falpha, fpalpha,
                                 lower, upper, order);
      }
      alpha_prev = alpha;
      falpha_prev = falpha;
      fpalpha_prev = fpalpha;
      alpha = alpha_next;
    }
    while (i++ < section_iters) {
      delta = b - a;
      {
        const double lower = a + tau2 * delta;
        const double upper = b - tau3 * delta;
        alpha = interpolate(a, fa, fpa, b, fb, fpb, lower, upper, order);
      }
      falpha = apply_f(alpha);
      if ((a - alpha) * fpa <= std::numeric_limits<double>::epsilon()) return kNoProgress;
      if (falpha > f0 + rho * alpha * fp0 || falpha >= fa) {
        b = alpha; fb = falpha; fpb = nan;
      } else {
        fpalpha = apply_df(alpha);
        if (std::fabs(fpalpha) <= -sigma * fp0) {
          alpha_new = alpha;
          return kSuccess;
        }
        if (((b - a) >= 0 && fpalpha >= 0) || ((b - a) <= 0 && fpalpha <= 0)) {
          b = a; fb = fa; fpb = fpa;
          a = alpha; fa = falpha; fpa = fpalpha;
        } else {
          a = alpha; fa = falpha; fpa = fpalpha;
        }
      }
    }
    return kSuccess;
  }
};

}  // namespace mgicp
