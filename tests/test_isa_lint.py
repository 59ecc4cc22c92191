"""CPU: the ISA lint over the product build's gfx950 code (scripts/isa_lint.py; hipcc
cross-compiles, no GPU): no wide LDS store has a data VGPR rewritten within 2 wait states, and
every M0-indexed register-image region of the tile pass holds only clamped 32-bit adds, with no LDS
load outstanding when a region opens (rule 4: LDS data returning under GPR-index mode lands outside
its destination — DESIGN.md §3, "Wide LDS stores" / "The tile-variant fault")."""

import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.exists(os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')) and not shutil.which('hipcc'),
                    reason='hipcc not available')
def test_isa_lint_product_build(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'scripts', 'isa_lint.py'), '--keep', str(tmp_path)],
                       capture_output=True, text=True, timeout=900)
    print(r.stdout[-3000:])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert 'isa lint: ok' in r.stdout
    # the lint saw the kernels it is about (a silently empty compile would pass trivially)
    assert 'nfi_render.hip: 0 wide' not in r.stdout
    assert 'M0-indexed regions, 0 violations' in r.stdout
