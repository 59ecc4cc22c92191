"""CPU: the ISA lint over the product build's gfx950 code (scripts/isa_lint.py; hipcc
cross-compiles, no GPU): no wide LDS store has a data VGPR rewritten within 2 wait states (rule 1),
no kernel uses GPR-index mode or M0-relative register moves (rule 2), and every indirect jump of the
assembled code object is a verified jump table of the tile pass — clamped slot, PC-relative target
that lands on the table, case k writing exactly image registers v(40+k), v(41+k), one exit (rule 6;
DESIGN.md §3).  The tile pass's integrity-check build (-DNFI_TILE_CHECK=1, loaded by
tests/test_gpu_tile_check.py) is linted the same way."""

import os
import re
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
    assert 'nfi_render.hip: 0 GPR-index-mode / movrel instructions' in r.stdout
    assert '16 jump tables, 0 violations' in r.stdout


def _lint_mod():
    import importlib.util
    spec = importlib.util.spec_from_file_location('isa_lint', os.path.join(ROOT, 'scripts', 'isa_lint.py'))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.skipif(not os.path.exists(os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')) and not shutil.which('hipcc'),
                    reason='hipcc not available')
def test_isa_lint_tilecheck_build(tmp_path):
    """the -DNFI_TILE_CHECK=1 library (extra loads, shuffles and a noinline failure call
    next to the tables) passes the same rules before tests/test_gpu_tile_check.py loads it."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'scripts', 'isa_lint.py'), '-D', 'NFI_TILE_CHECK=1',
                        os.path.join(ROOT, 'nerf-from-image_amd', 'csrc', 'nfi_render.hip')],
                       capture_output=True, text=True, timeout=900)
    print(r.stdout[-2000:])
    assert r.returncode == 0 and 'isa lint: ok' in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]
    assert '16 jump tables, 0 violations' in r.stdout


def _fn(body_lines, start=0x1000):
    """Synthetic llvm-objdump text: one function of (mnemonic + operands) lines, 4 bytes each (8 with
    a literal operand)."""
    out, addr = [f'{start:016x} <_Z1kv>:'], start
    for t in body_lines:
        size = 8 if re.search(r'\b(20|52)$', t) else 4
        tgt = ''
        m = re.match(r's_branch (\d+)$', t)
        if m:
            tgt = f' <_Z1kv+0x{addr + 4 + 4 * int(m.group(1)) - start:x}>'
        out.append(f'\t{t:58s} // {addr:012X}: 00000000{tgt}')
        addr += size
    return '\n'.join(out) + '\n'


def _table(case_reg=lambda k: 40 + k, clamp='s_min_u32 s0, s0, 30', off=20):
    body = ['s_and_b32 s0, s1, 31', clamp, 's_getpc_b64 s[88:89]', f's_lshl4_add_u32 s90, s0, {off}',
            's_add_u32 s88, s88, s90', 's_addc_u32 s89, s89, 0', 's_setpc_b64 s[88:89]']
    for k in range(31):
        r = case_reg(k)
        # 4 + 4 + 4 + 4 = 16 B per case; the branch skips the rest of the table to the exit
        body += [f'v_fmac_f32_e32 v{r}, v76, v117', f'v_fmac_f32_e32 v{r + 1}, s2, v76',
                 f's_branch {1 + 4 * (30 - k)}' if k < 30 else 's_branch 1', 's_nop 0']
    body += ['s_endpgm']
    return body


def test_rule6_jump_tables_synthetic():
    """Rule 6 on synthetic disassembly: the product's table verifies; a case writing the wrong image
    register, a missing slot clamp, a table offset that does not land on the table, and an indirect
    jump that is not a table are each reported."""
    lint = _lint_mod()
    n, bad = lint.jump_tables(_fn(_table()))
    assert n == 1 and not bad, bad
    n, bad = lint.jump_tables(_fn(_table(case_reg=lambda k: 40 + k + (k == 7))))
    assert bad and 'case 7' in bad[0][2]
    n, bad = lint.jump_tables(_fn(_table(clamp='s_min_u32 s0, s0, 31')))
    assert bad and 'not clamped' in bad[0][2]
    n, bad = lint.jump_tables(_fn(_table(off=52)))
    assert bad and 'table base' in bad[0][2]
    n, bad = lint.jump_tables(_fn(['s_load_dwordx2 s[4:5], s[0:1], 0x0', 's_setpc_b64 s[4:5]', 's_endpgm']))
    assert bad and 'not a table dispatch' in bad[0][2]
    n, bad = lint.jump_tables(_fn(['s_setpc_b64 s[30:31]']))      # a function return
    assert n == 0 and not bad


def test_rule2_no_index_mode(tmp_path):
    lint = _lint_mod()
    p = tmp_path / 'k.s'
    p.write_text('_Z1kv:\n\ts_set_gpr_idx_on s5, gpr_idx(SRC0,DST)\n\tv_add_f32 v40, v40, v2\n'
                 '\ts_set_gpr_idx_off\n\tv_movrels_b32 v1, v2\n\ts_endpgm\n')
    assert len(lint.no_index_mode(str(p))) == 3
    p.write_text('_Z1kv:\n\tv_add_f32 v40, v40, v2\n\ts_endpgm\n')
    assert not lint.no_index_mode(str(p))
