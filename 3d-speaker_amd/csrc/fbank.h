// Fbank tables + launcher (see fbank.hip).
#pragma once
#include "common.h"

namespace spk {

// Constant tables in double precision: the kernel computes the whole front end in fp64
// (feature noise is amplified ~60x into the embedding, so the fp32 FFT
// noise of a direct implementation would eat most of the 1e-4 embedding budget).
struct FbankTables {
  double window[400];       // Povey window hann(400, periodic=False)^0.85
  double2 twiddle[512];     // exp(-2 pi i j / 512), j = 0..511
  int mel_start[128];       // first FFT bin of filter m
  int mel_len[128];         // number of bins with non-zero weight
  int mel_off[128];         // offset of its weights in mel_w
  double mel_w[4096];
  int mel_nb;               // max mel_len rounded up to a multiple of 16
  int mel_blk_nb[4];        // max mel_len over bands 32 b .. 32 b + 31, rounded up to a multiple of 4
  double mel_wt[4096];      // dense zero-padded bank [t][m] = weight of bin mel_start[m] + t for
                            // band m, t < mel_nb: a wave's lanes (consecutive bands) read one line
};

// Host-side construction (double precision).  Returns the number of mel weights used;
// -1 if n_mels is unsupported.
int build_fbank_tables(FbankTables* t, int n_mels, double sample_rate);

// t_max > 0: utterance u is written at rows [u * t_max, u * t_max + frames_u), the rest of
// its t_max rows zeroed (a padded [n_utt, t_max, n_mels] batch); frame_off still gives frames_u
hipError_t launch_fbank(const float* wav, const int64_t* wav_off, int n_utt, float* feats,
                        const int64_t* frame_off, int n_mels, int mean_nor, const FbankTables* tab,
                        int mel_nb, hipStream_t s, int t_max = 0);

}  // namespace spk
