#pragma once
// Fused AFF module (speakerlab/models/eres2net/fusion.py:8-28) for the ERes2Net(V2)
// in-block fusions: one kernel instead of two 1x1 convs.  Channels-last [M, C] operands.
#include <string>

#include "common.h"

namespace spk {

struct AffDesc {
  const float* x = nullptr; int ldx = 0;      // AFF(x, y): x = previous split, y = this split
  const float* y = nullptr; int ldy = 0;
  float* out = nullptr; int ldo = 0;
  int M = 0;                                  // pixels (img, h, w)
  int cp = 0;                                 // channels of x, y and out (physical = logical)
  int nmid = 0;                               // bottleneck channels incl. zero padding (32 or 64)
  // local_att.0 (+ local_att.1 BN folded): [nmid][kp1] over K = 2*cp ([x | y]), bias [nmid]
  const float* w1 = nullptr; const uint16_t* w1h = nullptr; const uint16_t* w1l = nullptr;
  const float* b1 = nullptr; int kp1 = 0;
  // local_att.3 (+ local_att.4 BN folded): [cp][kp2] over K = nmid, bias [cp]
  const float* w2 = nullptr; const uint16_t* w2h = nullptr; const uint16_t* w2l = nullptr;
  const float* b2 = nullptr; int kp2 = 0;
  int* range_flag = nullptr;                  // fp16x3 range guard (common.h)
};

// true when launch_aff_x3 serves this geometry (fp16x3 path on, nmid 32 / 64, cp % 8 == 0)
bool aff_x3_supported(int cp, int nmid);
hipError_t launch_aff_x3(const AffDesc& a, hipStream_t s);
std::string aff_x3_kernel_name(int cp, int nmid);

}  // namespace spk
