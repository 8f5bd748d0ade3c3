// Probe kernel of tools/overlap_probe.py (diagnostic, not part of libebert): each workgroup
// records the XCD it runs on (HW_REG_XCC_ID) and its HW_ID (CU / SE fields), so that a CU-masked
// stream's bits can be mapped to XCDs. Built as a code object:
//   hipcc --offload-arch=gfx950 --genco tools/hw_probe.hip -o _abl/hw_probe.co
#include <hip/hip_runtime.h>
extern "C" __global__ void hw_probe(unsigned* out) {
  unsigned x, h;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(h));
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = x;
    out[2 * blockIdx.x + 1] = h;
  }
}
