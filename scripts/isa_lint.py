"""ISA lint over the gfx950 code of nfi's HIP sources (CPU only; hipcc cross-compiles).

Rule ("LDS rows written with kept-alive 32-bit stores"): a wide LDS store
(ds_write_b64 / b96 / b128, ds_write2_b32 / b64 and their st64 forms) reads its data VGPRs after
issue; an instruction that WRITES one of those VGPRs within WINDOW wait states after the store (one per
instruction, N + 1 for an s_nop N) can race with that read.  hipcc's hazard recognizer pads this for VMEM / FLAT stores wider than 8 bytes
but models no DS data hazard, and it does not look inside inline asm at all.  The lint lists every
wide DS store whose data registers are rewritten within WINDOW instructions (straight-line order;
labels do not stop the scan, an unconditional branch or s_endpgm does), says whether the writer sits
inside an inline-asm block (;;#ASMSTART .. ;;#ASMEND), and exits 1 if any is found.
Rule 2 (no_index_mode): no GPR-index mode (s_set_gpr_idx_*) and no M0-relative register moves
(v_movrel*, s_movrel*) anywhere in the build.  Round 5 measured register writes returning while
index mode was on land outside their destination (scripts/ubench/gpr_idx_probe.hip patterns 15, 16,
19: LDS returns, VALU-written index SGPRs, scalar-load returns); from round 6 the tile
pass's register image is updated through jump tables instead, and no kernel uses index mode.
Rule 6 (jump_tables): every indirect jump (s_setpc_b64) of the build other than a function return
is a jump table of the tile pass (nfi_render.hip tile_entry), checked on the ASSEMBLED code object
(llvm-objdump of the gfx950 ELF): s_getpc_b64 P; s_lshl4_add_u32 T, S, OFF; s_add_u32 P.lo, P.lo, T;
s_addc_u32 P.hi, P.hi, 0; s_setpc_b64 P — the slot SGPR S last written by s_min_u32 S, X, 30 before
it (so the jump stays inside the table); getpc's PC + OFF is the address right after the s_setpc;
case k (k = 0..30) at table + 16 k is v_fmac_f32 v(40+k) then v_fmac_f32 v(41+k) (the register
image's two texels of slot k) and an s_branch to the one exit, which lies after case 30.

Usage: python scripts/isa_lint.py [--window N] [--keep DIR] [source.hip ...]
(default: every nfi_*.hip in nerf-from-image_amd/csrc, compiled exactly as nfi/build.py compiles them,
with --cuda-device-only -S: the assembler text of the code object the product library carries).
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, 'nerf-from-image_amd', 'csrc')
sys.path.insert(0, os.path.join(ROOT, 'nerf-from-image_amd'))

WIDE_DS = re.compile(r'^\s*(ds_write(?:_b64|_b96|_b128|2_b32|2_b64|2st64_b32|2st64_b64))\s+(.*)$')
INSN = re.compile(r'^\s*([a-z_][a-z0-9_]*)(?:\s+(.*))?$')
VREG = re.compile(r'\bv(\d+)\b|\bv\[(\d+):(\d+)\]')
# instructions whose first operand is NOT a VGPR destination
NO_VDST = re.compile(r'^(ds_write|ds_store|global_store|buffer_store|flat_store|scratch_store|s_|v_cmp_|v_cmpx_|'
                     r'v_readlane|v_readfirstlane|ds_add_|ds_min_|ds_max_|ds_and_|ds_or_|ds_xor_|ds_inc_|'
                     r'ds_dec_|ds_cmpst|ds_nop|exp\b|buffer_wbl2|buffer_inv|global_atomic|buffer_atomic)')
STOP = re.compile(r'^\s*(s_branch|s_endpgm|s_setpc_b64)\b')


def regs(text: str) -> set[int]:
    out = set()
    for m in VREG.finditer(text):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def split_ops(s: str) -> list[str]:
    ops, depth, cur = [], 0, ''
    for ch in s:
        if ch == '[':
            depth += 1
        elif ch == ']':
            depth -= 1
        if ch == ',' and depth == 0:
            ops.append(cur.strip())
            cur = ''
        else:
            cur += ch
    if cur.strip():
        ops.append(cur.strip())
    return ops


def vdst(mnem: str, rest: str) -> set[int]:
    """VGPRs an instruction writes (its first operand, for the opcodes that have a VGPR destination)."""
    if NO_VDST.match(mnem) or not rest:
        return set()
    if mnem.startswith('ds_') and ('_rtn' not in mnem and not mnem.startswith(('ds_read', 'ds_load', 'ds_bpermute',
                                                                              'ds_permute', 'ds_swizzle'))):
        return set()
    first = split_ops(rest)[0]
    return regs(first) if first.startswith('v') else set()


def lint_asm(path: str, window: int):
    findings = []
    kernel = None
    lines = open(path).read().splitlines()
    in_asm = [False] * len(lines)
    state = False
    for i, ln in enumerate(lines):
        if ';;#ASMSTART' in ln:
            state = True
        elif ';;#ASMEND' in ln:
            state = False
        in_asm[i] = state
    loc = None
    files = {}
    for i, ln in enumerate(lines):
        if re.match(r'^_Z\S+:', ln):
            kernel = ln.split(':')[0]
        fm = re.match(r'^\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', ln)
        if fm:
            files[fm.group(1)] = os.path.basename(fm.group(3) or fm.group(2))
        lm = re.match(r'^\s*\.loc\s+(\d+)\s+(\d+)', ln)
        if lm:
            loc = f"{files.get(lm.group(1), lm.group(1))}:{lm.group(2)}"
        m = WIDE_DS.match(ln)
        if not m:
            continue
        ops = split_ops(m.group(2))
        data = set()
        for op in ops[1:]:
            if op.startswith('v'):
                data |= regs(op)
        if m.group(1) in ('ds_write_b64',) and not data:
            continue
        n = 0
        j = i + 1
        while j < len(lines) and n < window:
            t = lines[j].split(';')[0].rstrip()
            j += 1
            if not t.strip() or t.strip().endswith(':') or t.strip().startswith('.'):
                continue
            im = INSN.match(t)
            if not im:
                continue
            w = vdst(im.group(1), im.group(2) or '') & data
            n += 1
            if im.group(1) == 's_nop':   # s_nop N = N + 1 wait states
                n += int((im.group(2) or '0').strip(), 0)
            if w:
                findings.append({'kernel': kernel, 'line': i + 1, 'src': loc, 'store': ln.strip(), 'writer_line': j,
                                 'writer': t.strip(), 'distance': n, 'writer_in_inline_asm': in_asm[j - 1],
                                 'store_in_inline_asm': in_asm[i]})
                break
            if STOP.match(t):
                break
    return findings


INDEX_MODE = re.compile(r'^\s*(s_set_gpr_idx_\w+|v_movrel\w*|s_movrel\w*)\b')


def no_index_mode(path: str):
    """Rule 2: (kernel, line, instruction) of every GPR-index-mode / M0-relative register instruction
    in an assembler text file (there must be none)."""
    out, kernel = [], None
    for i, ln in enumerate(open(path).read().splitlines()):
        if re.match(r'^_Z\S+:', ln):
            kernel = ln.split(':')[0]
        if INDEX_MODE.match(ln.split(';')[0]):
            out.append((kernel, i + 1, ln.strip()))
    return out


DIS_FN = re.compile(r'^([0-9a-f]+) <(\S+)>:')
DIS_INS = re.compile(r'^\s+([a-z_0-9]+)(?:\s+([^/]*?))?\s*//\s*([0-9A-F]+):')


def parse_disassembly(text: str):
    """llvm-objdump -d text -> {function: [(address, mnemonic, operands)]} (branch operands as
    objdump prints them, with the absolute target appended as <fn+0xOFF>)."""
    fns, cur = {}, None
    for ln in text.splitlines():
        m = DIS_FN.match(ln)
        if m:
            cur = fns.setdefault(m.group(2), [])
            continue
        m = DIS_INS.match(ln)
        if m and cur is not None:
            ops = (m.group(2) or '').strip()
            t = re.search(r'<(\S+)\+0x([0-9a-f]+)>', ln)
            cur.append((int(m.group(3), 16), m.group(1), ops, (t.group(1), int(t.group(2), 16)) if t else None))
    starts = {}
    for ln in text.splitlines():
        m = DIS_FN.match(ln)
        if m:
            starts[m.group(2)] = int(m.group(1), 16)
    return fns, starts


CASE_BYTES, CASES, IMG_BASE = 16, 31, 40


def jump_tables(text: str):
    """Rule 6 over llvm-objdump text: returns (number of tables checked, [(function, address, message)])."""
    fns, starts = parse_disassembly(text)
    bad, checked = [], 0
    for fn, ins in fns.items():
        at = {a: j for j, (a, _, _, _) in enumerate(ins)}
        for jj, (saddr, smn, sops, _) in enumerate(ins):
            # every indirect jump: a function return (s[30:31], set by the caller's s_swappc_b64) or a
            # table dispatch, which must verify below
            if smn != 's_setpc_b64' or sops == 's[30:31]':
                continue
            checked += 1
            j = jj - 4
            if j < 0 or ins[j][1] != 's_getpc_b64' or ins[j][2] != sops:
                bad.append((fn, saddr, f'indirect jump s_setpc_b64 {sops} is not a table dispatch'))
                continue
            addr, mn, ops = ins[j][0], ins[j][1], ins[j][2]
            err = lambda msg: bad.append((fn, addr, msg))
            seq = ins[j + 1:j + 5]
            if [x[1] for x in seq] != ['s_lshl4_add_u32', 's_add_u32', 's_addc_u32', 's_setpc_b64']:
                err('not the table dispatch sequence: ' + ' ; '.join(f'{x[1]} {x[2]}' for x in seq))
                continue
            pm = re.match(r's\[(\d+):(\d+)\]$', ops)
            sh = [o.strip() for o in seq[0][2].split(',')]
            lo = [o.strip() for o in seq[1][2].split(',')]
            hi = [o.strip() for o in seq[2][2].split(',')]
            tmp, slot = sh[0], sh[1]
            ok = (pm and len(sh) == 3 and lo == [f's{pm.group(1)}', f's{pm.group(1)}', tmp]
                  and hi == [f's{pm.group(2)}', f's{pm.group(2)}', '0'] and seq[3][2] == ops)
            if not ok:
                err('dispatch operands do not form PC + (slot << 4) + OFF: ' + ' ; '.join(f'{x[1]} {x[2]}' for x in seq))
                continue
            try:
                off = int(sh[2], 0)
            except ValueError:
                err(f'table offset is not a literal: {sh[2]}')
                continue
            base = seq[0][0] + off            # s_getpc_b64 returns the address of the next instruction
            if j + 5 >= len(ins) or ins[j + 5][0] != base:
                err(f'table base {base:#x} is not the instruction after s_setpc_b64')
                continue
            # the slot SGPR's last write before the dispatch: s_min_u32 slot, X, 30
            clamp = None
            for q in range(j - 1, max(-1, j - 64), -1):
                qm, qo = ins[q][1], [o.strip() for o in ins[q][2].split(',')]
                if qm.startswith('s_') and not qm.startswith(('s_cmp', 's_bitcmp', 's_cbranch', 's_waitcnt', 's_nop',
                                                              's_branch', 's_setprio', 's_barrier')) and qo and qo[0] == slot:
                    clamp = (qm, qo)
                    break
            if not clamp or clamp[0] != 's_min_u32' or clamp[1][2:] != ['30']:
                err(f'slot {slot} not clamped to 30 by s_min_u32 before the dispatch (last write: {clamp})')
                continue
            exits = set()
            for k in range(CASES):
                c = at.get(base + CASE_BYTES * k)
                if c is None or c + 2 >= len(ins):
                    err(f'case {k}: no instruction at {base + CASE_BYTES * k:#x}')
                    break
                f0, f1, br = ins[c], ins[c + 1], ins[c + 2]
                fmac = ('v_fmac_f32', 'v_fmac_f32_e32')
                d0 = f0[2].split(',')[0].strip() if f0[1] in fmac else None
                d1 = f1[2].split(',')[0].strip() if f1[1] in fmac else None
                want0, want1 = f'v{IMG_BASE + k}', f'v{IMG_BASE + k + 1}'
                if (d0, d1) != (want0, want1) or br[1] != 's_branch' or br[3] is None:
                    err(f'case {k}: expected v_fmac_f32 {want0}; v_fmac_f32 {want1}; s_branch — got '
                        f'{f0[1]} {f0[2]} ; {f1[1]} {f1[2]} ; {br[1]} {br[2]}')
                    break
                exits.add(starts[br[3][0]] + br[3][1])
            else:
                end = base + CASE_BYTES * (CASES - 1)
                if len(exits) != 1 or not (end < next(iter(exits)) <= end + CASE_BYTES):
                    err(f'cases do not branch to one exit after the table: {sorted(hex(e) for e in exits)}')
    return checked, bad


def disassemble(src: str, extra=()):
    """llvm-objdump text of src's gfx950 code object, compiled as nfi/build.py compiles it."""
    from nfi.build import FLAGS
    flags = [f for f in FLAGS if f not in ('-shared', '-fPIC')]
    with tempfile.TemporaryDirectory() as d:
        obj = os.path.join(d, 'k.o')
        subprocess.run([os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')] + flags + ['-w', '--cuda-device-only',
                        '--no-gpu-bundle-output', '-c', '-o', obj, src] + list(extra), check=True)
        objdump = os.path.join(os.path.dirname(os.path.realpath(os.environ.get('HIPCC', '/opt/rocm/bin/hipcc'))), '..',
                               'lib', 'llvm', 'bin', 'llvm-objdump')
        if not os.path.exists(objdump):
            objdump = '/opt/rocm/lib/llvm/bin/llvm-objdump'
        return subprocess.run([objdump, '-d', '--mcpu=gfx950', obj], check=True, capture_output=True, text=True).stdout


DS_ANY = re.compile(r'^\s*(ds_(?:write|read|bpermute|permute|add|swizzle)\w*)\s+(.*)$')


def ds_addr_rewrites(path: str, window: int = 2, kernel_re: str = ''):
    """Report-only rule 3: DS instructions (stores, loads, permutes) whose ADDRESS VGPR an
    instruction rewrites within `window` wait states after issue — the address-side analogue of
    rule 1, the one pattern round 4's padded tile layout added to the tile pass's staging store
    (DESIGN.md §3).  Not a documented hazard (rule 1's data hazard was found by measurement); listed
    so a layout change that introduces one is visible in review.  Returns (kernel, line, insn, writer)."""
    out = []
    lines = open(path).read().splitlines()
    kernel = None
    for i, ln in enumerate(lines):
        if re.match(r'^_Z\S+:', ln):
            kernel = ln.split(':')[0]
        if kernel_re and not (kernel and re.search(kernel_re, kernel)):
            continue
        m = DS_ANY.match(ln.split(';')[0])
        if not m:
            continue
        ops = split_ops(m.group(2))
        mnem = m.group(1)
        # address = first operand for stores / atomics without return, second for loads and permutes
        aidx = 1 if mnem.startswith(('ds_read', 'ds_bpermute', 'ds_permute', 'ds_swizzle')) or '_rtn' in mnem else 0
        if len(ops) <= aidx or not ops[aidx].startswith('v'):
            continue
        addr = regs(ops[aidx])
        n, j = 0, i + 1
        while j < len(lines) and n < window:
            t = lines[j].split(';')[0].rstrip()
            j += 1
            if not t.strip() or t.strip().endswith(':') or t.strip().startswith('.'):
                continue
            im = INSN.match(t)
            if not im:
                continue
            n += 1
            if im.group(1) == 's_nop':
                n += int((im.group(2) or '0').strip(), 0)
            if vdst(im.group(1), im.group(2) or '') & addr:
                out.append((kernel, i + 1, ln.strip(), t.strip()))
                break
            if STOP.match(t):
                break
    return out


def compile_asm(src: str, out: str, extra=()):
    from nfi.build import FLAGS
    flags = [f for f in FLAGS if f not in ('-shared', '-fPIC')]
    cmd = [os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')] + flags + ['-w', '-gline-tables-only', '--cuda-device-only', '-S', '-o', out,
                                                                     src] + list(extra)
    subprocess.run(cmd, check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--window', type=int, default=2)
    ap.add_argument('--keep', default=None, help='directory to keep the .s files in')
    ap.add_argument('-D', action='append', default=[], help='extra -D defines (a variant build)')
    ap.add_argument('sources', nargs='*')
    a = ap.parse_args()
    srcs = a.sources or [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC)) if f.endswith('.hip')]
    tmp = a.keep or tempfile.mkdtemp(prefix='nfi_isa_')
    os.makedirs(tmp, exist_ok=True)
    total = []
    for s in srcs:
        out = os.path.join(tmp, os.path.basename(s).replace('.hip', '.s'))
        compile_asm(s, out, ['-D' + d for d in a.D])
        f = lint_asm(out, a.window)
        nstores = sum(1 for ln in open(out) if WIDE_DS.match(ln))
        print(f'{os.path.basename(s)}: {nstores} wide DS stores, {len(f)} with a data VGPR rewritten within '
              f'{a.window} instructions')
        for x in f:
            print(f"  {x['kernel'][:70]}  line {x['line']} ({x['src']}): {x['store']}\n"
                  f"      -> +{x['distance']} {x['writer']}"
                  f"{'  [writer inside inline asm]' if x['writer_in_inline_asm'] else ''}")
        total += f
        g = no_index_mode(out)
        print(f'{os.path.basename(s)}: {len(g)} GPR-index-mode / movrel instructions')
        for k, ln, msg in g:
            print(f'  {k[:70]}  line {ln}: {msg}')
        total += g
        if 'tile_entry' in open(s).read():
            n, jt = jump_tables(disassemble(s, ['-D' + d for d in a.D]))
            print(f'{os.path.basename(s)}: {n} jump tables, {len(jt)} violations')
            for fn, ad, msg in jt:
                print(f'  {fn[:70]}  {ad:#x}: {msg}')
            total += jt
            if n == 0:
                print('  (no jump table found: the tile pass was not compiled?)')
                total.append(('', 0, 'no jump table'))
    print('isa lint:', 'FAIL' if total else 'ok')
    return 1 if total else 0


if __name__ == '__main__':
    sys.exit(main())
