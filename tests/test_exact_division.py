"""The fast exact divisions used by the HIP kernels (grid_amd/csrc/common.hpp)
are bit-identical to IEEE division: q/100 EXHAUSTIVELY over every int32, and
the Markstein-corrected x/b over a large randomised sweep.  Compiled with gcc
and run on the CPU (IEEE fma is the same operation on gfx950)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SRC = r"""
#include <stdio.h>
#include <math.h>
#include <stdint.h>
#define __host__
#define __device__
#include "exact_div_only.h"
static inline uint64_t mix(uint64_t z){z+=0x9E3779B97F4A7C15ull;z=(z^(z>>30))*0xBF58476D1CE4E5B9ull;z=(z^(z>>27))*0x94D049BB133111EBull;return z^(z>>31);}
int main(void){
  long long bad = 0, bad2 = 0;
  #pragma omp parallel for reduction(+:bad)
  for (long long q = -2147483648LL; q <= 2147483647LL; q++)
    if (div100_exact((int32_t)q) != (double)q / 100.0) bad++;
  #pragma omp parallel for reduction(+:bad2)
  for (long long t = 0; t < 200000000LL; t++) {
    uint64_t h = mix(t), h2 = mix(h);
    double x = (double)(long long)(h % 4000000ull) / 100.0 * ((t & 2) ? -1.0 : 1.0);
    double b = 0.01 + (double)(h2 >> 11) * (1.0 / 9007199254740992.0) * 500.0;
    if (t % 3 == 0) b = sqrt(b);
    double r = 1.0 / b;
    if (div_exact(x, b, r) != x / b) bad2++;
  }
  printf("%lld %lld\n", bad, bad2);
  return 0;
}
"""


def test_exact_division_identities(tmp_path):
    if not shutil.which("gcc"):
        pytest.skip("gcc not available")
    hdr = open(os.path.join(ROOT, "grid_amd", "csrc", "common.hpp")).read()
    body = hdr[hdr.index("// ---- exact fast division"):]
    if "// ---- compact depth matrix" in body:
        body = body[: body.index("// ---- compact depth matrix")]
    (tmp_path / "exact_div_only.h").write_text("#include <math.h>\n#include <stdint.h>\n" +
                                              body.replace("inline", "static inline"))
    (tmp_path / "t.c").write_text(SRC)
    exe = tmp_path / "t"
    subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", "-o", str(exe), str(tmp_path / "t.c"),
                    "-I", str(tmp_path), "-lm"], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True, timeout=600).stdout.split()
    assert out == ["0", "0"], out
