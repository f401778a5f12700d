// Test infrastructure only (oracle): a C entry point over the REFERENCE's own image-method generator
// (create_data/rirgen.cpp:115-351, compiled from /root/reference by oracle/Makefile into oracle/_ref/),
// so tests can compare sepvad_rir_generate with it bit for bit. Mirrors the pyrirgen.generateRir call
// the reference's data pipeline makes (create_data/pyrirgen.pyx, create_simulation_data.py:284-289).
#include <vector>

std::vector<std::vector<double> > gen_rir(double c, double fs, const std::vector<std::vector<double> >& rr,
                                          const std::vector<double>& ss, const std::vector<double>& LL,
                                          const std::vector<double>& beta_input, const std::vector<double>& orientation,
                                          int isHighPassFilter, int nDimension, int nOrder, int nSamples,
                                          char microphone_type);

extern "C" int ref_rir_generate(double c, double fs, const double* mics, int n_mics, const double* src,
                                const double* room, const double* beta, int n_beta, const double* orientation,
                                int high_pass, int n_dim, int order, int n_samples, char mic_type, double* out,
                                long long cap) {
  std::vector<std::vector<double> > rr(n_mics, std::vector<double>(3));
  for (int m = 0; m < n_mics; ++m)
    for (int i = 0; i < 3; ++i) rr[m][i] = mics[3 * m + i];
  std::vector<double> ss(src, src + 3), LL(room, room + 3), bb(beta, beta + n_beta);
  std::vector<double> oo(orientation, orientation + 2);
  std::vector<std::vector<double> > h = gen_rir(c, fs, rr, ss, LL, bb, oo, high_pass, n_dim, order, n_samples, mic_type);
  const int n = h.empty() ? 0 : (int)h[0].size();
  if ((long long)n_mics * n > cap) return -1;
  for (int m = 0; m < n_mics; ++m)
    for (int i = 0; i < n; ++i) out[(long long)m * n + i] = h[m][i];
  return n;
}
