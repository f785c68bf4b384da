// Host construction of the Fbank constant tables (double precision, kept in double).
// Window: torchaudio _feature_window_function(POVEY) = hann_window(400, periodic=False)^0.85.
// Mel bank: torchaudio get_mel_banks (mel = 1127 ln(1 + f/700), low 20 Hz, high = Nyquist,
// 512-point FFT, vtln_warp = 1), the Nyquist column is zero so only bins 0..255 carry weight.
#include <algorithm>
#include <cmath>
#include "fbank.h"

namespace spk {

int build_fbank_tables(FbankTables* t, int n_mels, double sample_rate) {
  if (n_mels <= 3 || n_mels > 128) return -1;
  const double pi = 3.14159265358979323846;
  for (int i = 0; i < 400; ++i) {
    const double h = 0.5 - 0.5 * std::cos(2.0 * pi * i / 399.0);
    t->window[i] = std::pow(h, 0.85);
  }
  for (int k = 0; k < 512; ++k) {
    const double a = -2.0 * pi * k / 512.0;
    t->twiddle[k] = make_double2(std::cos(a), std::sin(a));
  }
  auto mel = [](double f) { return 1127.0 * std::log(1.0 + f / 700.0); };
  const double nyq = 0.5 * sample_rate;
  const double bin_w = sample_rate / 512.0;
  const double mlo = mel(20.0), mhi = mel(nyq);
  const double delta = (mhi - mlo) / (n_mels + 1);
  int off = 0, maxlen = 0;
  for (int m = 0; m < n_mels; ++m) {
    const double left = mlo + m * delta, center = mlo + (m + 1) * delta, right = mlo + (m + 2) * delta;
    int first = -1, last = -1;
    for (int b = 0; b < 256; ++b) {
      const double mb = mel(bin_w * b);
      const double w = std::fmax(0.0, std::fmin((mb - left) / (center - left), (right - mb) / (right - center)));
      if (w > 0.0) {
        if (first < 0) first = b;
        last = b;
      }
    }
    if (first < 0) { first = 0; last = -1; }
    t->mel_start[m] = first;
    t->mel_len[m] = last - first + 1;
    maxlen = std::max(maxlen, last - first + 1);
    t->mel_off[m] = off;
    for (int b = first; b <= last; ++b) {
      const double mb = mel(bin_w * b);
      const double w = std::fmax(0.0, std::fmin((mb - left) / (center - left), (right - mb) / (right - center)));
      if (off >= 4096) return -1;
      t->mel_w[off++] = w;
    }
  }
  t->mel_nb = (maxlen + 15) / 16 * 16;
  for (int b = 0; b < 4; ++b) {
    int mx = 0;
    for (int m = 32 * b; m < std::min(n_mels, 32 * b + 32); ++m) mx = std::max(mx, t->mel_len[m]);
    t->mel_blk_nb[b] = (mx + 3) / 4 * 4;
  }
  if (t->mel_nb * n_mels > 4096) return -1;
  for (int i = 0; i < t->mel_nb * n_mels; ++i) {
    const int tt = i / n_mels, m = i - tt * n_mels;
    t->mel_wt[i] = tt < t->mel_len[m] ? t->mel_w[t->mel_off[m] + tt] : 0.0;
  }
  return off;
}

}  // namespace spk
