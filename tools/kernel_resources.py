"""Per-kernel VGPR/AGPR/spill/LDS/occupancy table from hipcc's resource-usage remarks.

Usage: python tools/kernel_resources.py 3d-speaker_amd/csrc/conv_gemm.hip [more.hip ...]
"""
import os
import re
import subprocess
import sys

CSRC = '3d-speaker_amd/csrc'


def main():
    for src in sys.argv[1:]:
        p = subprocess.run(['hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '-I', CSRC, '-c', src] + os.environ.get('KR_FLAGS', '').split() + [
                            '-o', '/dev/null', '-Rpass-analysis=kernel-resource-usage'],
                           capture_output=True, text=True)
        cur = None
        rows = []
        for line in p.stderr.splitlines():
            m = re.search(r'remark: (?:.*?: )?\s*([A-Za-z /\[\]]+?): (\S+) \[-Rpass', line)
            if not m:
                continue
            k, v = m.group(1).strip(), m.group(2)
            if k == 'Function Name':
                cur = {'name': subprocess.run(['c++filt', v], capture_output=True, text=True).stdout.strip()}
                rows.append(cur)
            elif cur is not None:
                cur[k] = v
        for r in rows:
            name = re.sub(r'^(void )?spk::(\(anonymous namespace\)::)?', '', r['name'])
            name = re.sub(r'\(.*\)$', '', name)
            print(f"{r.get('VGPRs', '?'):>4} v {r.get('AGPRs', '?'):>3} a  spill {r.get('VGPRs Spill', '?'):>3}  "
                  f"lds {int(r.get('LDS Size [bytes/block]', 0)) // 1024:>3} KB  occ {r.get('Occupancy [waves/SIMD]', '?'):>2}  "
                  f"{name}")


if __name__ == '__main__':
    main()
