// Image-method room impulse responses (Allen & Berkley 1979; Peterson 1986), host side: the generator the
// reference's data pipeline calls through pyrirgen.generateRir (create_data/rirgen.cpp:115-351,
// create_data/create_simulation_data.py:284-289) to make the reverberant mixtures of BASELINE cfg 4.
//
// Restated from the published algorithm as the reference implements it (same loop nest and the same
// double-precision operation order per contribution, so results match it bit for bit; tests compare
// with the reference compiled from its own source into oracle/_ref):
//   * T60 -> reflection coefficients by Sabine: alpha = 24 V ln10 / (c S T60), beta = sqrt(1 - alpha)
//     (T60 = 0: anechoic, beta = 0); nsamples = T60 fs by default (from the betas when given: Sabine's
//     T60, at least 0.128 s);
//   * positions in units of c/fs; for every image (mx, my, mz) in the +-ceil(n/(2L)) lattice and every
//     mirror (q, j, k): distance, reflection gain prod beta^|m-q| beta^|m|, microphone directivity,
//     1 / (4 pi d c/fs), and a fractional-delay Hann-windowed sinc of width Tw = 2 round(0.004 fs);
//   * optional Allen-Berkley high-pass (100 Hz two-pole) in place.
#include <cmath>
#include <cstdlib>
#include <vector>

#include "../../include/sepvad.h"

namespace {

constexpr double kPi = 3.14159265358979323846;

long round_half_away(double x) { return x >= 0 ? (long)(x + 0.5) : (long)(x - 0.5); }

double sinc_d(double x) { return x == 0 ? 1.0 : std::sin(x) / x; }

// Polar-pattern gain of a directional microphone (rho: b 0, h 0.25, c 0.5, s 0.75; omni: 1).
double mic_gain(double x, double y, double z, const double* angle, char mtype) {
  double rho;
  switch (mtype) {
    case 'b': rho = 0.0; break;
    case 'h': rho = 0.25; break;
    case 'c': rho = 0.5; break;
    case 's': rho = 0.75; break;
    default: return 1.0;
  }
  const double vartheta = std::acos(z / std::sqrt(std::pow(x, 2) + std::pow(y, 2) + std::pow(z, 2)));
  const double varphi = std::atan2(y, x);
  double gain = std::sin(kPi / 2 - angle[1]) * std::sin(vartheta) * std::cos(angle[0] - varphi) +
                std::cos(kPi / 2 - angle[1]) * std::cos(vartheta);
  return rho + (1 - rho) * gain;
}

}  // namespace

extern "C" int32_t sepvad_rir_generate(double c, double fs, const double* mics, int32_t n_mics, const double* src,
                                       const double* room, const double* beta_in, int32_t n_beta,
                                       const double* orientation, int32_t high_pass, int32_t n_dim, int32_t order,
                                       int32_t n_samples, char mic_type, double* out, int64_t cap) {
  if (!mics || !src || !room || !beta_in || n_mics < 1 || (n_beta != 1 && n_beta != 6) || c <= 0 || fs <= 0)
    return SEPVAD_E_ARG;
  double beta[6];
  double t60 = 0.0;
  if (n_beta == 1) {
    const double V = room[0] * room[1] * room[2];
    const double S = 2 * (room[0] * room[2] + room[1] * room[2] + room[0] * room[1]);
    t60 = beta_in[0];
    if (t60 != 0) {
      const double alfa = 24 * V * std::log(10.0) / (c * S * t60);
      for (double& b : beta) b = std::sqrt(1 - alfa);
    } else {
      for (double& b : beta) b = 0;
    }
  } else {
    for (int i = 0; i < 6; ++i) beta[i] = beta_in[i];
  }
  const double angle[2] = {orientation ? orientation[0] : 0.0, orientation ? orientation[1] : 0.0};
  if (n_dim == 2) beta[4] = beta[5] = 0;
  if (n_samples == -1) {
    if (n_beta > 1) {
      const double V = room[0] * room[1] * room[2];
      const double alpha = ((1 - std::pow(beta[0], 2)) + (1 - std::pow(beta[1], 2))) * room[1] * room[2] +
                           ((1 - std::pow(beta[2], 2)) + (1 - std::pow(beta[3], 2))) * room[0] * room[2] +
                           ((1 - std::pow(beta[4], 2)) + (1 - std::pow(beta[5], 2))) * room[0] * room[1];
      t60 = 24 * std::log(10.0) * V / (c * alpha);
      if (t60 < 0.128) t60 = 0.128;
    }
    n_samples = (int)(t60 * fs);
  }
  if (n_samples < 0) return SEPVAD_E_ARG;
  if (!out) return n_samples;  // size query
  if (cap < (int64_t)n_mics * n_samples) return SEPVAD_E_ARG;

  const int Tw = 2 * (int)round_half_away(0.004 * fs);
  const double cTs = c / fs, Fc = 1.0;
  const double s[3] = {src[0] / cTs, src[1] / cTs, src[2] / cTs};
  const double L[3] = {room[0] / cTs, room[1] / cTs, room[2] / cTs};
  std::vector<double> lpi(Tw);
  // high-pass filter constants (cut-off 100 Hz)
  const double W = 2 * kPi * 100 / fs, R1 = std::exp(-W), B1 = 2 * R1 * std::cos(W), B2 = -R1 * R1, A1 = -(1 + R1);

  for (int im = 0; im < n_mics; ++im) {
    double* h = out + (size_t)im * n_samples;
    for (int i = 0; i < n_samples; ++i) h[i] = 0.0;
    const double r[3] = {mics[3 * im] / cTs, mics[3 * im + 1] / cTs, mics[3 * im + 2] / cTs};
    const int n1 = (int)std::ceil(n_samples / (2 * L[0]));
    const int n2 = (int)std::ceil(n_samples / (2 * L[1]));
    const int n3 = (int)std::ceil(n_samples / (2 * L[2]));
    for (int mx = -n1; mx <= n1; ++mx) {
      const double Rmx = 2 * mx * L[0];
      for (int my = -n2; my <= n2; ++my) {
        const double Rmy = 2 * my * L[1];
        for (int mz = -n3; mz <= n3; ++mz) {
          const double Rmz = 2 * mz * L[2];
          for (int q = 0; q <= 1; ++q) {
            const double px = (1 - 2 * q) * s[0] - r[0] + Rmx;
            const double gx = std::pow(beta[0], std::abs(mx - q)) * std::pow(beta[1], std::abs(mx));
            for (int j = 0; j <= 1; ++j) {
              const double py = (1 - 2 * j) * s[1] - r[1] + Rmy;
              const double gy = std::pow(beta[2], std::abs(my - j)) * std::pow(beta[3], std::abs(my));
              for (int k = 0; k <= 1; ++k) {
                const double pz = (1 - 2 * k) * s[2] - r[2] + Rmz;
                const double gz = std::pow(beta[4], std::abs(mz - k)) * std::pow(beta[5], std::abs(mz));
                const double dist = std::sqrt(std::pow(px, 2) + std::pow(py, 2) + std::pow(pz, 2));
                if (!(std::abs(2 * mx - q) + std::abs(2 * my - j) + std::abs(2 * mz - k) <= order || order == -1)) continue;
                const double fdist = std::floor(dist);
                if (!(fdist < n_samples)) continue;
                const double gain = mic_gain(px, py, pz, angle, mic_type) * gx * gy * gz / (4 * kPi * dist * cTs);
                for (int n = 0; n < Tw; ++n)
                  lpi[n] = 0.5 * (1 - std::cos(2 * kPi * ((n + 1 - (dist - fdist)) / Tw))) * Fc *
                           sinc_d(kPi * Fc * (n + 1 - (dist - fdist) - (Tw / 2)));
                const int start = (int)fdist - (Tw / 2) + 1;
                for (int n = 0; n < Tw; ++n)
                  if (start + n >= 0 && start + n < n_samples) h[start + n] += gain * lpi[n];
              }
            }
          }
        }
      }
    }
    if (high_pass == 1) {
      double y0 = 0, y1 = 0, y2 = 0;
      for (int i = 0; i < n_samples; ++i) {
        const double x0 = h[i];
        y2 = y1;
        y1 = y0;
        y0 = B1 * y1 + B2 * y2 + x0;
        h[i] = y0 + A1 * y1 + R1 * y2;
      }
    }
  }
  return n_samples;
}
