// ORACLE (test infrastructure only): C entry point around the REFERENCE's own radix-2 FFT
// (runtime/onnxruntime/feature/feature_functions.cpp:17-60), compiled from the reference
// sources where they lie by oracle/Makefile into oracle/_ref/libref_fft.so.  Used by
// tests/test_fbank_oracle.py to pin the FFT step of the numpy Fbank oracle.
#include <complex>
#include <vector>

#include "feature/feature_functions.h"

extern "C" int ref_custom_fft(const float* re_in, const float* im_in, int n, float* re_out, float* im_out) {
  if (n <= 0 || (n & (n - 1))) return -1;
  std::vector<int> bitrev;
  std::vector<float> sintbl;
  speakerlab::init_bit_reverse_index(bitrev, n);
  speakerlab::init_sin_tbl(sintbl, n);
  std::vector<std::complex<float>> d(n);
  for (int i = 0; i < n; ++i) d[i] = std::complex<float>(re_in[i], im_in ? im_in[i] : 0.f);
  speakerlab::custom_fft(bitrev, sintbl, d);
  for (int i = 0; i < n; ++i) {
    re_out[i] = d[i].real();
    im_out[i] = d[i].imag();
  }
  return 0;
}
