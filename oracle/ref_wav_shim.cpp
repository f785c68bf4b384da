// ORACLE (test infrastructure only): C entry points around the REFERENCE's own runtime WAV
// reader (runtime/onnxruntime/utils/wav_reader.cpp:7-57, compiled from the reference sources
// where they lie by oracle/Makefile into oracle/_ref/libref_wav.so), and the std::ostream
// float formatting its embedding writer uses (bin/extract_speaker_embedding.cpp:54-69).
// Used by tests/test_runtime_io.py to pin speakerlab/utils/runtime_io.py.
#include <cstring>
#include <sstream>
#include <string>
#include <vector>

#include "utils/wav_reader.h"

extern "C" int ref_read_wav(const char* path, float* out, int max_n, int* n, int* sr, int* nch, int* nsample) {
  speakerlab::WavReader r{std::string(path)};
  if (!r.is_valid()) return -1;
  const std::vector<float> v = r.get_float_wav_data();
  *n = (int)v.size();
  *sr = (int)r.sample_rate();
  *nch = r.num_channel();
  *nsample = (int)r.num_sample();
  for (int i = 0; i < (int)v.size() && i < max_n; ++i) out[i] = v[i];
  return 0;
}

extern "C" int ref_format_float(float v, char* buf, int len) {
  std::ostringstream s;
  s << v;
  const std::string t = s.str();
  if ((int)t.size() + 1 > len) return -1;
  std::memcpy(buf, t.c_str(), t.size() + 1);
  return 0;
}
