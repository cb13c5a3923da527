// ORACLE / CPU BASELINE — test and measurement infrastructure only; never linked into,
// loaded by or called from the product path (hmsc_amd/).
//
// A compiled C++ restatement of the reference's Gibbs sweep for the BASELINE config-4 class
// (R/sampleMcmc.R:219-306 with C = NULL, one non-spatial random level, no NA, probit and
// normal species; updateGammaEta off as SURVEY.md §8(d) prescribes for the timed run), used as
// bench.py's `cpu_baseline` ("Fallback if R is absent: time the build's C++ CPU
// restatement, single-threaded per chain, chains = cores").  It follows oracle/hmsc_oracle.py
// function by function (each cites the R lines it restates) and shares its randomness
// contract (oracle/rng.py: Philox4x32-10, AS241 quantile, libm erfc / log), so a chain here
// equals the numpy oracle's up to floating-point rounding (tests/test_oracle_cpu_port.py).
//
// Layout: every ny-long vector is a contiguous column (X, XEta, Z, S column-major), so the
// ny x ns x K contractions of a sweep are axpy / dot loops the compiler vectorises.
//
//   build (oracle/cpu_port.py; AVX2 + FMA, runs on any current x86 host): g++ -O3 -march=x86-64-v3 -fPIC -shared -pthread oracle/cpu/hmsc_cpu.cpp -o oracle/libhmsc_cpu.so
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace {

// ------------------------------- randomness (oracle/rng.py) -------------------------------
enum Stream : uint32_t {
  S_GAMMA2 = 1, S_BETALAMBDA = 3, S_WISHART_DIAG = 4, S_WISHART_OFF = 5, S_GAMMAV = 6, S_INVSIGMA = 11, S_Z = 12,
  S_PSI = 20, S_DELTA = 21, S_ETA = 22, S_INIT_GAMMA = 40, S_INIT_V_DIAG = 41, S_INIT_V_OFF = 42,
  S_INIT_BETA = 43, S_INIT_SIGMA = 44, S_INIT_DELTA = 50, S_INIT_PSI = 51, S_INIT_LAMBDA = 52, S_INIT_ETA = 53,
};
constexpr uint32_t GAMMA_BOOST_SUB = 0xFFFF0000u;
constexpr int GAMMA_MAX_TRIALS = 64;

struct Rng {
  uint32_t k0, k1;
  explicit Rng(uint64_t seed) : k0((uint32_t)(seed & 0xFFFFFFFFu)), k1((uint32_t)(seed >> 32)) {}
  void words(uint32_t idx, uint32_t sub, uint32_t stream, uint32_t it, uint32_t w[4]) const {
    uint32_t c0 = idx, c1 = sub, c2 = stream, c3 = it, q0 = k0, q1 = k1;
    for (int r = 0; r < 10; ++r) {
      const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
      const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ q0, n1 = (uint32_t)p1;
      const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ q1, n3 = (uint32_t)p0;
      c0 = n0, c1 = n1, c2 = n2, c3 = n3;
      q0 += 0x9E3779B9u;
      q1 += 0xBB67AE85u;
    }
    w[0] = c0, w[1] = c1, w[2] = c2, w[3] = c3;
  }
  void block(uint32_t idx, uint32_t sub, uint32_t stream, uint32_t it, double* a, double* b) const {
    uint32_t w[4];
    words(idx, sub, stream, it, w);
    *a = ((double)(w[0] >> 5) * 67108864.0 + (double)(w[1] >> 6) + 0.5) * (1.0 / 9007199254740992.0);
    *b = ((double)(w[2] >> 5) * 67108864.0 + (double)(w[3] >> 6) + 0.5) * (1.0 / 9007199254740992.0);
  }
  double uniform(uint32_t idx, uint32_t sub, uint32_t stream, uint32_t it) const {
    double a, b;
    block(idx, sub, stream, it, &a, &b);
    return a;
  }
  double normal(uint32_t idx, uint32_t sub, uint32_t stream, uint32_t it) const;
  double gamma_std(uint32_t idx, uint32_t stream, uint32_t it, double shape) const;
  double gamma(uint32_t idx, uint32_t stream, uint32_t it, double shape, double rate) const {
    return gamma_std(idx, stream, it, shape) / rate;
  }
};

double qnorm_as241(double p) {  // Wichura AS241 PPND16 (R's qnorm)
  const double q = p - 0.5;
  if (std::fabs(q) <= 0.425) {
    const double r = 0.180625 - q * q;
    const double num = (((((((2.5090809287301226727e+3 * r + 3.3430575583588128105e+4) * r + 6.7265770927008700853e+4) * r +
                            4.5921953931549871457e+4) * r + 1.3731693765509461125e+4) * r + 1.9715909503065514427e+3) * r +
                         1.3314166789178437745e+2) * r + 3.3871328727963666080e0);
    const double den = (((((((5.2264952788528545610e+3 * r + 2.8729085735721942674e+4) * r + 3.9307895800092710610e+4) * r +
                            2.1213794301586595867e+4) * r + 5.3941960214247511077e+3) * r + 6.8718700749205790830e+2) * r +
                         4.2313330701600911252e+1) * r + 1.0);
    return q * num / den;
  }
  double r = std::sqrt(-std::log(q < 0.0 ? p : 1.0 - p));
  double val;
  if (r <= 5.0) {
    r -= 1.6;
    const double num = (((((((7.74545014278341407640e-4 * r + 2.27238449892691845833e-2) * r + 2.41780725177450611770e-1) * r +
                            1.27045825245236838258e0) * r + 3.64784832476320460504e0) * r + 5.76949722146069140550e0) * r +
                         4.63033784615654529590e0) * r + 1.42343711074968357734e0);
    const double den = (((((((1.05075007164441684324e-9 * r + 5.47593808499534494600e-4) * r + 1.51986665636164571966e-2) * r +
                            1.48103976427480074590e-1) * r + 6.89767334985100004550e-1) * r + 1.67638483018380384940e0) * r +
                         2.05319162663775882187e0) * r + 1.0);
    val = num / den;
  } else {
    r -= 5.0;
    const double num = (((((((2.01033439929228813265e-7 * r + 2.71155556874348757815e-5) * r + 1.24266094738807843860e-3) * r +
                            2.65321895265761230930e-2) * r + 2.96560571828504891230e-1) * r + 1.78482653991729133580e0) * r +
                         5.46378491116411436990e0) * r + 6.65790464350110377720e0);
    const double den = (((((((2.04426310338993978564e-15 * r + 1.42151175831644588870e-7) * r + 1.84631831751005468180e-5) * r +
                            7.86869131145613259100e-4) * r + 1.48753612908506148525e-2) * r + 1.36929880922735805310e-1) * r +
                         5.99832206555887937690e-1) * r + 1.0);
    val = num / den;
  }
  return q < 0.0 ? -val : val;
}

double Rng::normal(uint32_t idx, uint32_t sub, uint32_t stream, uint32_t it) const {
  return qnorm_as241(uniform(idx, sub, stream, it));
}

double Rng::gamma_std(uint32_t idx, uint32_t stream, uint32_t it, double shape) const {  // Marsaglia-Tsang
  const double a = shape < 1.0 ? shape + 1.0 : shape;
  const double d = a - 1.0 / 3.0, c = 1.0 / std::sqrt(9.0 * d);
  double out = d;
  for (int t = 0; t < GAMMA_MAX_TRIALS; ++t) {
    const double x = normal(idx, 2u * t, stream, it);
    double v = 1.0 + c * x;
    if (v <= 0.0) continue;
    v = v * v * v;
    const double u = uniform(idx, 2u * t + 1u, stream, it);
    if (std::log(u) < 0.5 * x * x + d - d * v + d * std::log(v)) {
      out = d * v;
      break;
    }
  }
  if (shape < 1.0) out *= std::pow(uniform(idx, GAMMA_BOOST_SUB, stream, it), 1.0 / shape);
  return out;
}

double trunc_normal_lower(double alpha, double u) {  // oracle/rng.py trunc_normal_lower
  if (alpha > 25.0) return alpha - std::log(u) / alpha;
  return -qnorm_as241(u * (0.5 * std::erfc(alpha * 0.7071067811865476)));
}

// ------------------------------- small dense algebra (column-major) -------------------------------
using Mat = std::vector<double>;

// upper R with R'R = A (R's chol)
Mat chol_upper(const Mat& A, int n) {
  Mat R(n * n, 0.0);
  for (int j = 0; j < n; ++j) {
    double d = A[j + n * j];
    for (int k = 0; k < j; ++k) d -= R[k + n * j] * R[k + n * j];
    if (!(d > 0.0)) throw std::runtime_error("chol: matrix not positive definite");
    d = std::sqrt(d);
    R[j + n * j] = d;
    for (int i = j + 1; i < n; ++i) {
      double v = A[j + n * i];
      for (int k = 0; k < j; ++k) v -= R[k + n * j] * R[k + n * i];
      R[j + n * i] = v / d;
    }
  }
  return R;
}
Mat transpose(const Mat& A, int m, int n) {  // A m x n -> n x m
  Mat T((size_t)m * n);
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < m; ++i) T[j + (size_t)n * i] = A[i + (size_t)m * j];
  return T;
}
// x <- R^-1 x (backsolve) / R^-T x (backsolve(..., transpose = TRUE)), R upper
void backsolve(const Mat& R, int n, double* x) {
  for (int i = n - 1; i >= 0; --i) {
    double s = x[i];
    for (int k = i + 1; k < n; ++k) s -= R[i + n * k] * x[k];
    x[i] = s / R[i + n * i];
  }
}
void backsolve_t(const Mat& R, int n, double* x) {
  for (int i = 0; i < n; ++i) {
    double s = x[i];
    for (int k = 0; k < i; ++k) s -= R[k + n * i] * x[k];
    x[i] = s / R[i + n * i];
  }
}
Mat chol2inv(const Mat& R, int n) {  // (R'R)^-1
  Mat Inv(n * n, 0.0), e(n);
  for (int c = 0; c < n; ++c) {
    std::fill(e.begin(), e.end(), 0.0);
    e[c] = 1.0;
    backsolve_t(R, n, e.data());
    backsolve(R, n, e.data());
    for (int i = 0; i < n; ++i) Inv[i + n * c] = e[i];
  }
  return Inv;
}
Mat inv_spd(const Mat& A, int n) { return chol2inv(chol_upper(A, n), n); }
Mat mm(const Mat& A, const Mat& B, int m, int k, int n) {  // (m x k)(k x n)
  Mat C((size_t)m * n, 0.0);
  for (int j = 0; j < n; ++j)
    for (int q = 0; q < k; ++q) {
      const double b = B[q + (size_t)k * j];
      for (int i = 0; i < m; ++i) C[i + (size_t)m * j] += A[i + (size_t)m * q] * b;
    }
  return C;
}
Mat kron(const Mat& A, int ma, int na, const Mat& B, int mb, int nb) {
  const int m = ma * mb, n = na * nb;
  Mat K((size_t)m * n);
  for (int ja = 0; ja < na; ++ja)
    for (int jb = 0; jb < nb; ++jb)
      for (int ia = 0; ia < ma; ++ia)
        for (int ib = 0; ib < mb; ++ib)
          K[(ia * mb + ib) + (size_t)m * (ja * nb + jb)] = A[ia + (size_t)ma * ja] * B[ib + (size_t)mb * jb];
  return K;
}
Mat eye(int n) {
  Mat I(n * n, 0.0);
  for (int i = 0; i < n; ++i) I[i + n * i] = 1.0;
  return I;
}

// MCMCpack::rwish restated (oracle rwish): Bartlett construction with upper Z
Mat rwish(double v, const Mat& S, int p, const Rng& rng, uint32_t it, uint32_t s_diag, uint32_t s_off) {
  const Mat CC = chol_upper(S, p);
  Mat Zm(p * p, 0.0);
  for (int i = 0; i < p; ++i) Zm[i + p * i] = std::sqrt(2.0 * rng.gamma_std(i, s_diag, it, (v - i) / 2.0));
  for (int b = 1; b < p; ++b)
    for (int a = 0; a < b; ++a) Zm[a + p * b] = rng.normal(a + p * b, 0, s_off, it);
  const Mat ZC = mm(Zm, CC, p, p, p);
  return mm(transpose(ZC, p, p), ZC, p, p, p);
}

// ------------------------------- model and chain state -------------------------------
struct Model {
  int ny, ns, nc, nt, np, nf;
  const double *X, *Y, *Yraw, *Tr;  // ny x nc, ny x ns (YScaled, hM$Y), ns x nt (column-major)
  const int* Pi;               // ny, 1-based unit of each row
  const int* fam;              // ns: 1 normal, 2 probit
  const int* varest;           // ns: distr[, 2]
  Mat V0, UGamma, mGamma, aSigma, bSigma;
  double f0, nu, a1, b1, a2, b2;
};

struct Chain {
  const Model& m;
  Rng rng;
  int K;
  Mat Gamma, iV, Beta, iSigma, Eta, Lambda, Psi, Delta, Z;  // Eta np x nf, Lambda nf x ns
  Mat XEta, E, S;                                           // ny x K, ny work columns
  Chain(const Model& mm_, uint64_t seed) : m(mm_), rng(seed), K(mm_.nc + mm_.nf) {}

  void build_xeta() {  // R/updateBetaLambda.R:21-41
    const int ny = m.ny, nc = m.nc;
    XEta.assign((size_t)ny * K, 0.0);
    std::memcpy(XEta.data(), m.X, sizeof(double) * ny * nc);
    for (int h = 0; h < m.nf; ++h)
      for (int i = 0; i < ny; ++i) XEta[i + (size_t)ny * (nc + h)] = Eta[(m.Pi[i] - 1) + (size_t)m.np * h];
  }

  // updateZ, R/updateZ.R:4-94 (normal :40-41, probit :43-63); Y = hM$Y at init
  void update_z(uint32_t it, bool raw_y = false) {
    const int ny = m.ny;
    build_xeta();
    std::vector<double> e(ny), ua(ny), ub(ny);
    for (int j = 0; j < m.ns; ++j) {
      double* zc = &Z[(size_t)ny * j];
      const double* yc = (raw_y ? m.Yraw : m.Y) + (size_t)ny * j;
      if (m.fam[j] == 1) {
        std::memcpy(zc, yc, sizeof(double) * ny);
        continue;
      }
      std::fill(e.begin(), e.end(), 0.0);
      for (int c = 0; c < m.nc; ++c) {
        const double b = Beta[c + (size_t)m.nc * j];
        const double* x = &XEta[(size_t)ny * c];
        for (int i = 0; i < ny; ++i) e[i] += x[i] * b;
      }
      for (int h = 0; h < m.nf; ++h) {
        const double l = Lambda[h + (size_t)m.nf * j];
        const double* x = &XEta[(size_t)ny * (m.nc + h)];
        for (int i = 0; i < ny; ++i) e[i] += x[i] * l;
      }
      const double sd = 1.0 / std::sqrt(iSigma[j]);
      for (int i = 0; i < ny; ++i) {  // one Philox block per (site, species quad), word j & 3
        uint32_t q[4];
        rng.words(i + (uint32_t)ny * (uint32_t)(j >> 2), 0, S_Z, it, q);
        const double u = ((double)q[j & 3] + 0.5) * (1.0 / 4294967296.0);
        const double s = yc[i] == 1.0 ? 1.0 : -1.0;
        const double w = trunc_normal_lower(-s * e[i] / sd, u);
        zc[i] = e[i] + sd * s * w;
      }
    }
  }

  void init() {  // computeInitialParameters, R/computeInitialParameters.R:17-273 (initPar = NULL)
    const int nc = m.nc, nt = m.nt, ns = m.ns, N = nc * nt, nf = m.nf;
    const uint32_t it = 0;
    Mat LU = transpose(chol_upper(m.UGamma, N), N, N);  // lower
    Gamma.assign(N, 0.0);
    for (int a = 0; a < N; ++a) {
      double v = m.mGamma[a];
      for (int b = 0; b < N; ++b) v += LU[a + N * b] * rng.normal(b, 0, S_INIT_GAMMA, it);
      Gamma[a] = v;
    }
    const Mat V = inv_spd(rwish(m.f0, inv_spd(m.V0, nc), nc, rng, it, S_INIT_V_DIAG, S_INIT_V_OFF), nc);  // :91
    iV = inv_spd(V, nc);
    const Mat LV = transpose(chol_upper(V, nc), nc, nc);
    Beta.assign((size_t)nc * ns, 0.0);
    std::vector<double> xi(nc);
    for (int j = 0; j < ns; ++j) {  // :97-101
      for (int k = 0; k < nc; ++k) xi[k] = rng.normal(j, k, S_INIT_BETA, it);
      for (int c = 0; c < nc; ++c) {
        double mu = 0.0;
        for (int t = 0; t < nt; ++t) mu += Gamma[c + nc * t] * m.Tr[j + (size_t)ns * t];
        for (int k = 0; k < nc; ++k) mu += LV[c + nc * k] * xi[k];
        Beta[c + (size_t)nc * j] = mu;
      }
    }
    iSigma.assign(ns, 1.0);  // :111-126
    for (int j = 0; j < ns; ++j)
      if (m.varest[j] == 1) iSigma[j] = 1.0 / rng.gamma(j, S_INIT_SIGMA, it, m.aSigma[j], m.bSigma[j]);
    Delta.assign(nf, 0.0);  // :156-200, level 0
    Delta[0] = rng.gamma(0, S_INIT_DELTA, it, m.a1, m.b1);
    for (int h = 1; h < nf; ++h) Delta[h] = rng.gamma(h, S_INIT_DELTA, it, m.a2, m.b2);
    Psi.assign((size_t)nf * ns, 0.0);
    Lambda.assign((size_t)nf * ns, 0.0);
    std::vector<double> tau(nf);
    double c = 1.0;
    for (int h = 0; h < nf; ++h) tau[h] = (c *= Delta[h]);
    for (int j = 0; j < ns; ++j)
      for (int h = 0; h < nf; ++h) {
        const double psi = rng.gamma(h + nf * j, S_INIT_PSI, it, m.nu / 2, m.nu / 2);
        Psi[h + (size_t)nf * j] = psi;
        Lambda[h + (size_t)nf * j] = rng.normal(h + nf * j, 0, S_INIT_LAMBDA, it) / std::sqrt(psi * tau[h]);
      }
    Eta.assign((size_t)m.np * nf, 0.0);  // :207
    for (int h = 0; h < nf; ++h)
      for (int q = 0; q < m.np; ++q) Eta[q + (size_t)m.np * h] = rng.normal(q, h, S_INIT_ETA, it);
    Z.assign((size_t)m.ny * ns, 0.0);
    update_z(0, true);  // :254 Z = updateZ(Y = hM$Y, ...)
  }

  bool all_unit_isigma() const {
    for (double v : iSigma)
      if (v != 1.0) return false;
    return true;
  }

  // updateGamma2, R/updateGamma2.R:6-60 (oracle gamma2_moments / update_gamma2)
  void update_gamma2(uint32_t it) {
    if (!all_unit_isigma()) return;  // :35-36
    const int ny = m.ny, nc = m.nc, nt = m.nt, ns = m.ns, N = nc * nt;
    build_xeta();
    // S Tr with S = Z - LRan (:20-33, :46): accumulate over species
    Mat ST((size_t)ny * nt, 0.0);
    std::vector<double> s(ny);
    for (int j = 0; j < ns; ++j) {
      std::memcpy(s.data(), &Z[(size_t)ny * j], sizeof(double) * ny);
      for (int h = 0; h < m.nf; ++h) {
        const double l = Lambda[h + (size_t)m.nf * j];
        const double* x = &XEta[(size_t)ny * (nc + h)];
        for (int i = 0; i < ny; ++i) s[i] -= x[i] * l;
      }
      for (int t = 0; t < nt; ++t) {
        const double tr = m.Tr[j + (size_t)ns * t];
        double* d = &ST[(size_t)ny * t];
        for (int i = 0; i < ny; ++i) d[i] += s[i] * tr;
      }
    }
    Mat XZT((size_t)nc * nt, 0.0), XX((size_t)nc * nc, 0.0), TT((size_t)nt * nt, 0.0);
    for (int t = 0; t < nt; ++t)
      for (int c = 0; c < nc; ++c) {
        double v = 0.0;
        for (int i = 0; i < ny; ++i) v += m.X[i + (size_t)ny * c] * ST[i + (size_t)ny * t];
        XZT[c + nc * t] = v;
      }
    for (int a = 0; a < nc; ++a)
      for (int b = 0; b < nc; ++b) {
        double v = 0.0;
        for (int i = 0; i < ny; ++i) v += m.X[i + (size_t)ny * a] * m.X[i + (size_t)ny * b];
        XX[a + nc * b] = v;
      }
    for (int a = 0; a < nt; ++a)
      for (int b = 0; b < nt; ++b) {
        double v = 0.0;
        for (int j = 0; j < ns; ++j) v += m.Tr[j + (size_t)ns * a] * m.Tr[j + (size_t)ns * b];
        TT[a + nt * b] = v;
      }
    const Mat iUG = inv_spd(m.UGamma, N);
    Mat iV0(nc * nc);
    for (int a = 0; a < nc; ++a)
      for (int b = 0; b < nc; ++b) iV0[a + nc * b] = iUG[a + N * b];  // :37
    const Mat V0 = inv_spd(iV0, nc);
    Mat iVXX(nc * nc);
    for (int q = 0; q < nc * nc; ++q) iVXX[q] = iV[q] + XX[q];
    const Mat iP = inv_spd(iVXX, nc);
    const Mat LiP = transpose(chol_upper(iP, nc), nc, nc);
    const Mat t1 = mm(iV, LiP, nc, nc, nc);
    const Mat t1t = mm(t1, transpose(t1, nc, nc), nc, nc, nc);
    Mat D(nc * nc);
    for (int q = 0; q < nc * nc; ++q) D[q] = iV[q] - t1t[q];
    Mat Rin = kron(eye(nt), nt, nt, iV0, nc, nc);
    const Mat k2 = kron(TT, nt, nt, D, nc, nc);
    for (size_t q = 0; q < Rin.size(); ++q) Rin[q] += k2[q];
    const Mat Rm = inv_spd(Rin, N);                                   // :44
    const Mat LR = transpose(chol_upper(Rm, N), N, N);
    const Mat iPXZT = mm(iP, XZT, nc, nc, nt);
    const Mat XXiPXZT = mm(XX, iPXZT, nc, nc, nt);
    const Mat V0XXiPiV = mm(mm(mm(V0, XX, nc, nc, nc), iP, nc, nc, nc), iV, nc, nc, nc);
    const Mat tmp = kron(TT, nt, nt, V0XXiPiV, nc, nc);
    Mat d1((size_t)nc * nt);
    for (int q = 0; q < nc * nt; ++q) d1[q] = XZT[q] - XXiPXZT[q];
    Mat muG = mm(V0, d1, nc, nc, nt);
    const Mat w = mm(tmp, mm(Rm, mm(iV, iPXZT, nc, nc, nt), N, N, 1), N, N, 1);
    for (int q = 0; q < N; ++q) muG[q] -= w[q];
    const Mat V0XXV0 = mm(mm(V0, XX, nc, nc, nc), V0, nc, nc, nc);  // V0 X'(V0 X')' without ny
    const Mat t2 = mm(mm(V0, XX, nc, nc, nc), LiP, nc, nc, nc);
    const Mat t2t = mm(t2, transpose(t2, nc, nc), nc, nc, nc);
    Mat Dm(nc * nc);
    for (int q = 0; q < nc * nc; ++q) Dm[q] = V0XXV0[q] - t2t[q];
    const Mat t3 = mm(tmp, LR, N, N, N);
    Mat SigmaG = kron(eye(nt), nt, nt, V0, nc, nc);                   // :50
    const Mat k3 = kron(TT, nt, nt, Dm, nc, nc);
    const Mat t3t = mm(t3, transpose(t3, N, N), N, N, N);
    for (size_t q = 0; q < SigmaG.size(); ++q) SigmaG[q] += t3t[q] - k3[q];
    const Mat LS = transpose(chol_upper(SigmaG, N), N, N);
    for (int a = 0; a < N; ++a) {                                     // :53-54
      double v = muG[a];
      for (int b = 0; b < N; ++b) v += LS[a + N * b] * rng.normal(b, 0, S_GAMMA2, it);
      Gamma[a] = v;
    }
  }

  // updateBetaLambda, C = NULL branch, no NA: R/updateBetaLambda.R:8-157
  void update_beta_lambda(uint32_t it) {
    const int ny = m.ny, nc = m.nc, ns = m.ns, nf = m.nf;
    build_xeta();
    Mat G((size_t)K * K);  // :65
    for (int a = 0; a < K; ++a)
      for (int b = a; b < K; ++b) {
        double v = 0.0;
        const double *x = &XEta[(size_t)ny * a], *y = &XEta[(size_t)ny * b];
        for (int i = 0; i < ny; ++i) v += x[i] * y[i];
        G[a + K * b] = G[b + K * a] = v;
      }
    std::vector<double> tau(nf);
    double c = 1.0;
    for (int h = 0; h < nf; ++h) tau[h] = (c *= Delta[h]);  // :51
    Mat P(K * K), iU(K * K);
    std::vector<double> rhs(K), mu(K), xs(K), xi(K);
    for (int j = 0; j < ns; ++j) {
      const double* zc = &Z[(size_t)ny * j];
      for (int k = 0; k < K; ++k) {  // :66 XEta' Z_j
        double v = 0.0;
        const double* x = &XEta[(size_t)ny * k];
        for (int i = 0; i < ny; ++i) v += x[i] * zc[i];
        xs[k] = v;
      }
      std::fill(P.begin(), P.end(), 0.0);
      for (int a = 0; a < nc; ++a)
        for (int b = 0; b < nc; ++b) P[a + K * b] = iV[a + nc * b];  // :83-89
      for (int h = 0; h < nf; ++h) P[(nc + h) * (K + 1)] = Psi[h + (size_t)nf * j] * tau[h];
      std::fill(mu.begin(), mu.end(), 0.0);
      for (int a = 0; a < nc; ++a)
        for (int t = 0; t < m.nt; ++t) mu[a] += Gamma[a + nc * t] * m.Tr[j + (size_t)ns * t];  // :62
      for (int q = 0; q < K * K; ++q) iU[q] = P[q] + G[q] * iSigma[j];  // :92
      for (int a = 0; a < K; ++a) {
        double v = xs[a] * iSigma[j];
        for (int b = 0; b < K; ++b) v += P[a + K * b] * mu[b];
        rhs[a] = v;
      }
      const Mat R = chol_upper(iU, K);  // :98
      backsolve_t(R, K, rhs.data());    // mean = R^-1 R^-T rhs ; draw mean + R^-1 xi   (:99-101)
      for (int k = 0; k < K; ++k) rhs[k] += rng.normal(j, k, S_BETALAMBDA, it);
      backsolve(R, K, rhs.data());
      for (int a = 0; a < nc; ++a) Beta[a + (size_t)nc * j] = rhs[a];
      for (int h = 0; h < nf; ++h) Lambda[h + (size_t)nf * j] = rhs[nc + h];
    }
  }

  // updateGammaV, R/updateGammaV.R:4-34 (C = NULL)
  void update_gamma_v(uint32_t it) {
    const int nc = m.nc, nt = m.nt, ns = m.ns, N = nc * nt;
    Mat E((size_t)nc * ns);
    for (int j = 0; j < ns; ++j)
      for (int a = 0; a < nc; ++a) {
        double v = Beta[a + (size_t)nc * j];
        for (int t = 0; t < nt; ++t) v -= Gamma[a + nc * t] * m.Tr[j + (size_t)ns * t];
        E[a + (size_t)nc * j] = v;
      }
    Mat A(nc * nc, 0.0);
    for (int a = 0; a < nc; ++a)
      for (int b = 0; b < nc; ++b) {
        double v = 0.0;
        for (int j = 0; j < ns; ++j) v += E[a + (size_t)nc * j] * E[b + (size_t)nc * j];
        A[a + nc * b] = v + m.V0[a + nc * b];
      }
    const Mat Vn = inv_spd(A, nc);                                     // :19
    iV = rwish(m.f0 + ns, Vn, nc, rng, it, S_WISHART_DIAG, S_WISHART_OFF);  // :20
    const Mat iUG = inv_spd(m.UGamma, N);
    Mat TT((size_t)nt * nt, 0.0);
    for (int a = 0; a < nt; ++a)
      for (int b = 0; b < nt; ++b) {
        double v = 0.0;
        for (int j = 0; j < ns; ++j) v += m.Tr[j + (size_t)ns * a] * m.Tr[j + (size_t)ns * b];
        TT[a + nt * b] = v;
      }
    Mat Pg = kron(TT, nt, nt, iV, nc, nc);
    for (size_t q = 0; q < Pg.size(); ++q) Pg[q] += iUG[q];
    const Mat RG = chol_upper(Pg, N);                                  // :29
    std::vector<double> rhs(N, 0.0);
    for (int a = 0; a < N; ++a)
      for (int b = 0; b < N; ++b) rhs[a] += iUG[a + N * b] * m.mGamma[b];
    for (int t = 0; t < nt; ++t)                                       // vec((iV Beta) Tr)
      for (int a = 0; a < nc; ++a) {
        double v = 0.0;
        for (int j = 0; j < ns; ++j) {
          double ib = 0.0;
          for (int b = 0; b < nc; ++b) ib += iV[a + nc * b] * Beta[b + (size_t)nc * j];
          v += ib * m.Tr[j + (size_t)ns * t];
        }
        rhs[a + nc * t] += v;
      }
    const Mat C = chol2inv(RG, N);
    std::vector<double> xi(N);
    for (int a = 0; a < N; ++a) xi[a] = rng.normal(a, 0, S_GAMMAV, it);
    backsolve(RG, N, xi.data());
    for (int a = 0; a < N; ++a) {                                      // :30-31
      double v = xi[a];
      for (int b = 0; b < N; ++b) v += C[a + N * b] * rhs[b];
      Gamma[a] = v;
    }
  }

  // updateLambdaPriors, R/updateLambdaPriors.R:3-53 (matrix branch :21-33)
  void update_lambda_priors(uint32_t it) {
    const int nf = m.nf, ns = m.ns;
    std::vector<double> tau(nf), rs(nf, 0.0);
    double c = 1.0;
    for (int h = 0; h < nf; ++h) tau[h] = (c *= Delta[h]);
    for (int j = 0; j < ns; ++j)
      for (int h = 0; h < nf; ++h) {
        const double l2 = Lambda[h + (size_t)nf * j] * Lambda[h + (size_t)nf * j];
        const double psi = rng.gamma(h + nf * j, S_PSI, it, m.nu / 2 + 0.5, m.nu / 2 + 0.5 * l2 * tau[h]);  // :22-23
        Psi[h + (size_t)nf * j] = psi;
        rs[h] += psi * l2;
      }
    double s = 0.0;
    for (int h = 0; h < nf; ++h) s += tau[h] * rs[h];
    Delta[0] = rng.gamma(0, S_DELTA, it, m.a1 + 0.5 * ns * nf, m.b1 + 0.5 * s / Delta[0]);  // :25-27
    for (int h = 1; h < nf; ++h) {  // :28-32
      c = 1.0;
      for (int q = 0; q < nf; ++q) tau[q] = (c *= Delta[q]);
      double b = 0.0;
      for (int q = h; q < nf; ++q) b += tau[q] * rs[q];
      Delta[h] = rng.gamma(h, S_DELTA, it, m.a2 + 0.5 * ns * (nf - h), m.b2 + 0.5 * b / Delta[h]);
    }
  }

  // updateEta, non-spatial level without NA: R/updateEta.R:42-92
  void update_eta(uint32_t it) {
    const int ny = m.ny, nc = m.nc, ns = m.ns, nf = m.nf, np = m.np;
    Mat bs((size_t)np * nf, 0.0);  // Ssum (Lambda diag(iSigma))'
    std::vector<double> s(ny);
    for (int j = 0; j < ns; ++j) {  // S = Z - X Beta (:31-37)
      std::memcpy(s.data(), &Z[(size_t)ny * j], sizeof(double) * ny);
      for (int c = 0; c < nc; ++c) {
        const double b = Beta[c + (size_t)nc * j];
        const double* x = m.X + (size_t)ny * c;
        for (int i = 0; i < ny; ++i) s[i] -= x[i] * b;
      }
      for (int h = 0; h < nf; ++h) {
        const double l = Lambda[h + (size_t)nf * j] * iSigma[j];
        double* d = &bs[(size_t)np * h];
        for (int i = 0; i < ny; ++i) d[m.Pi[i] - 1] += s[i] * l;
      }
    }
    Mat LL(nf * nf, 0.0);  // Lambda iSigma Lambda' (:45)
    for (int a = 0; a < nf; ++a)
      for (int b = 0; b < nf; ++b) {
        double v = 0.0;
        for (int j = 0; j < ns; ++j) v += Lambda[a + (size_t)nf * j] * iSigma[j] * Lambda[b + (size_t)nf * j];
        LL[a + nf * b] = v;
      }
    std::vector<int> nq(np, 0);
    for (int i = 0; i < ny; ++i) nq[m.Pi[i] - 1]++;
    Mat Q(nf * nf);
    std::vector<double> y(nf);
    int last_n = -1;
    Mat R;
    for (int q = 0; q < np; ++q) {  // :46-57, :72-91
      if (nq[q] != last_n) {
        for (int a = 0; a < nf * nf; ++a) Q[a] = LL[a] * nq[q] + (a % (nf + 1) == 0 ? 1.0 : 0.0);
        R = chol_upper(Q, nf);
        last_n = nq[q];
      }
      for (int h = 0; h < nf; ++h) y[h] = bs[q + (size_t)np * h];
      backsolve_t(R, nf, y.data());
      for (int h = 0; h < nf; ++h) y[h] += rng.normal(q, h, S_ETA, it);
      backsolve(R, nf, y.data());
      for (int h = 0; h < nf; ++h) Eta[q + (size_t)np * h] = y[h];
    }
  }

  // updateInvSigma, R/updateInvSigma.R:3-43 (species with distr[,2] == 1 only)
  void update_inv_sigma(uint32_t it) {
    const int ny = m.ny;
    bool any = false;
    for (int j = 0; j < m.ns; ++j) any |= m.varest[j] == 1;
    if (!any) return;
    build_xeta();
    for (int j = 0; j < m.ns; ++j) {
      if (m.varest[j] != 1) continue;
      double ss = 0.0;
      for (int i = 0; i < ny; ++i) {
        double e = Z[i + (size_t)ny * j];
        for (int c = 0; c < m.nc; ++c) e -= XEta[i + (size_t)ny * c] * Beta[c + (size_t)m.nc * j];
        for (int h = 0; h < m.nf; ++h) e -= XEta[i + (size_t)ny * (m.nc + h)] * Lambda[h + (size_t)m.nf * j];
        ss += e * e;
      }
      iSigma[j] = rng.gamma(j, S_INVSIGMA, it, m.aSigma[j] + ny / 2.0, m.bSigma[j] + ss / 2.0);  // :37-40
    }
  }

  void sweep(uint32_t it, bool gamma2) {  // R/sampleMcmc.R:219-306, updater GammaEta = FALSE
    if (gamma2) update_gamma2(it);
    update_beta_lambda(it);
    update_gamma_v(it);
    update_lambda_priors(it);
    update_eta(it);
    update_inv_sigma(it);  // Alpha: rep(1, nf) for a non-spatial level (R/updateAlpha.R:81-82)
    update_z(it);
  }
};

thread_local std::string g_err;

}  // namespace

extern "C" {

const char* hmsc_cpu_last_error(void) { return g_err.c_str(); }

// Model arrays column-major as R stores them.  priors = {f0, nu, a1, b1, a2, b2}.
// Runs `nchains` independent chains (seed + 7919 c) for `n_sweeps` sweeps after the initial
// state, each chain on its own thread; writes chain 0's final state to the out arrays (any
// may be NULL) and the wall time of the sweeps (init excluded) to *seconds.
int hmsc_cpu_run(int ny, int ns, int nc, int nt, int np, int nf, const double* X, const double* Y, const double* Yraw,
                 const double* Tr,
                 const int* Pi, const int* fam, const int* varest, const double* V0, const double* UGamma,
                 const double* mGamma, const double* aSigma, const double* bSigma, const double* priors,
                 uint64_t seed, int nchains, int n_sweeps, int iter0, int gamma2, double* Beta, double* Gamma,
                 double* iV, double* Lambda, double* Eta, double* Psi, double* Delta, double* Z, double* iSigma,
                 double* seconds) {
  try {
    Model m{};
    m.ny = ny, m.ns = ns, m.nc = nc, m.nt = nt, m.np = np, m.nf = nf;
    m.X = X, m.Y = Y, m.Yraw = Yraw ? Yraw : Y, m.Tr = Tr, m.Pi = Pi, m.fam = fam, m.varest = varest;
    const int N = nc * nt;
    m.V0.assign(V0, V0 + nc * nc);
    m.UGamma.assign(UGamma, UGamma + N * N);
    m.mGamma.assign(mGamma, mGamma + N);
    m.aSigma.assign(aSigma, aSigma + ns);
    m.bSigma.assign(bSigma, bSigma + ns);
    m.f0 = priors[0], m.nu = priors[1], m.a1 = priors[2], m.b1 = priors[3], m.a2 = priors[4], m.b2 = priors[5];
    for (int j = 0; j < ns; ++j)
      if (fam[j] != 1 && fam[j] != 2) throw std::runtime_error("hmsc_cpu: only normal and probit species");
    std::vector<Chain*> chains;
    for (int c = 0; c < nchains; ++c) chains.push_back(new Chain(m, seed + 7919ull * (uint64_t)c));
    std::vector<std::string> errs(nchains);
    auto init_all = [&](int c) {
      try {
        chains[c]->init();
      } catch (const std::exception& e) {
        errs[c] = e.what();
      }
    };
    auto run_all = [&](int c) {
      try {
        for (int k = 1; k <= n_sweeps; ++k) chains[c]->sweep((uint32_t)(iter0 + k), gamma2 != 0);
      } catch (const std::exception& e) {
        errs[c] = e.what();
      }
    };
    {
      std::vector<std::thread> th;
      for (int c = 0; c < nchains; ++c) th.emplace_back(init_all, c);
      for (auto& t : th) t.join();
    }
    const auto t0 = std::chrono::steady_clock::now();
    {
      std::vector<std::thread> th;
      for (int c = 0; c < nchains; ++c) th.emplace_back(run_all, c);
      for (auto& t : th) t.join();
    }
    const auto t1 = std::chrono::steady_clock::now();
    if (seconds) *seconds = std::chrono::duration<double>(t1 - t0).count();
    for (auto& e : errs)
      if (!e.empty()) throw std::runtime_error(e);
    const Chain& c0 = *chains[0];
    auto put = [](double* dst, const Mat& src) {
      if (dst) std::memcpy(dst, src.data(), sizeof(double) * src.size());
    };
    put(Beta, c0.Beta), put(Gamma, c0.Gamma), put(iV, c0.iV), put(Lambda, c0.Lambda), put(Eta, c0.Eta);
    put(Psi, c0.Psi), put(Delta, c0.Delta), put(Z, c0.Z), put(iSigma, c0.iSigma);
    for (auto* c : chains) delete c;
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

}  // extern "C"
