#pragma once
// Whole-block fusion of the ERes2NetV2 Res2Net bottleneck (speakerlab/models/eres2net/
// ERes2NetV2.py:65-91, BasicBlockERes2NetV2 with scale 2 and an identity shortcut):
//   conv1 1x1 + bn1 + Hardtanh -> split(width) -> sp = conv0(s0) ; sp1 = conv1(sp + s1)
//   (3x3 + bn + Hardtanh each) -> cat -> conv3 1x1 + bn3 + residual + Hardtanh
// in one persistent kernel per spatial tile: the conv1 output, the Res2Net slices and the
// concat never leave LDS, so a block moves its input and its output through HBM once.
#include <string>

#include "common.h"

namespace spk {

struct Res2Desc {
  const float* x = nullptr;     // block input (and residual), channels-last [nimg, H, W, C]
  float* out = nullptr;         // [nimg, H, W, Cout]
  int nimg = 0, H = 0, W = 0, C = 0;
  int Cout = 0;                 // output channels (0: C)
  int stride = 1;               // conv1 / shortcut stride; H, W are the OUTPUT dims, the input is
  int Hin = 0, Win = 0;         // [nimg, Hin, Win, C] (0: H, W); the stage-2 projection block uses 2
  bool proj = false;            // 1x1 projection shortcut + BN (ERes2NetV2.py:84-88), packed
                                // into w3 as K columns 64 .. 64+C, its BN shift into b3
  int width = 0;                // Res2Net slice width (26 for ERes2NetV2 layer1, 52 for layer2), <= 64
  // fp16 hi / lo planes of the BN-folded packed weights (Model::pack) and fp32 biases:
  const uint16_t* w1h = nullptr; const uint16_t* w1l = nullptr; const float* b1 = nullptr;   // [64][C]
  const uint16_t* wah = nullptr; const uint16_t* wal = nullptr; const float* ba = nullptr;   // convs.0 [32][9*32]
  const uint16_t* wbh = nullptr; const uint16_t* wbl = nullptr; const float* bb = nullptr;   // convs.1 [32][9*32]
  const uint16_t* w3h = nullptr; const uint16_t* w3l = nullptr; const float* b3 = nullptr;   // [Cout][64 (+C)]
  const float* w1 = nullptr; const float* wa = nullptr;   // the same four matrices in fp32 (the
  const float* wb = nullptr; const float* w3 = nullptr;   // host emulation of the kernel reads them)
};

bool res2_block_supported(const Res2Desc& d);
hipError_t launch_res2_block(const Res2Desc& d, hipStream_t s);
std::string res2_block_kernel_name(const Res2Desc& d);

}  // namespace spk
