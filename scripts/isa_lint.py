"""ISA lint over the gfx950 code of nfi's HIP sources (CPU only; hipcc cross-compiles).

Rule ("LDS rows written with kept-alive 32-bit stores"): a wide LDS store
(ds_write_b64 / b96 / b128, ds_write2_b32 / b64 and their st64 forms) reads its data VGPRs after
issue; an instruction that WRITES one of those VGPRs within WINDOW wait states after the store (one per
instruction, N + 1 for an s_nop N) can race with that read.  hipcc's hazard recognizer pads this for VMEM / FLAT stores wider than 8 bytes
but models no DS data hazard, and it does not look inside inline asm at all.  The lint lists every
wide DS store whose data registers are rewritten within WINDOW instructions (straight-line order;
labels do not stop the scan, an unconditional branch or s_endpgm does), says whether the writer sits
inside an inline-asm block (;;#ASMSTART .. ;;#ASMEND), and exits 1 if any is found.
Rule 2 (lint_gpr_idx): the M0-indexed register-image regions of the tile pass.
Rule 5 (valu_sgpr_near_region): no v_readfirstlane / v_readlane shortly before a region (probes 16-18).
Rule 4 (lds_return_in_region): no LDS load and no scalar load may be outstanding at an
s_set_gpr_idx_on — data returning while GPR-index mode is on corrupts registers outside its
destination (round 5: scripts/ubench/gpr_idx_probe.hip patterns 15 (LDS) and 19 (scalar) fault the
GPU; the same with a global load, pattern 14, is exact).

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


def lint_gpr_idx(path: str):
    """Rule 2 (the tile pass's register image, nfi_render.hip img_add / img_fma2): every M0-indexed
    region (s_set_gpr_idx_on .. s_set_gpr_idx_off) holds only 32-bit VOP2 v_add_f32 vD, vD, vX under
    gpr_idx(SRC0,DST) on the pinned image base vD = v40 / v41 (no packed or 64-bit operand: an odd
    index would address an unaligned VGPR pair; no VOP3 form: a VOP3 v_fma_f32 under gpr_idx(SRC2,DST)
    broke the pass on MI355X), and
    its index SGPR was clamped to <= 30 by an s_min just before (v40 + 31 + 1 = v72 is outside the
    image), so no index reaches past v71."""
    bad = []
    lines = open(path).read().splitlines()
    kernel = None
    for i, ln in enumerate(lines):
        if re.match(r'^_Z\S+:', ln):
            kernel = ln.split(':')[0]
        m = re.match(r'^\s*s_set_gpr_idx_on\s+(s\d+)', ln)
        if not m:
            continue
        idx = m.group(1)
        prev = [x.split(';')[0].strip() for x in lines[max(0, i - 30):i]]
        prev = [x for x in prev if x and not x.startswith('.') and not x.endswith(':')]
        if not any(re.match(rf's_min_[iu]32\s+{idx},\s*{idx},\s*30$', x) or
                   re.match(rf's_min_[iu]32\s+{idx},\s*s\d+,\s*30$', x) for x in prev):
            bad.append((kernel, i + 1, f'index {idx} not clamped to 30 before the region'))
        j = i + 1
        while j < len(lines) and 's_set_gpr_idx_off' not in lines[j]:
            t = lines[j].split(';')[0].strip()
            j += 1
            if not t or t.startswith('.'):
                continue
            mode = re.search(r'gpr_idx\(([A-Z0-9,]+)\)', ln)
            mode = mode.group(1) if mode else ''
            ok_add = mode == 'SRC0,DST' and re.match(r'v_add_f32(_e32)?\s+(v4[01]),\s*\2,\s*v\d+$', t)
            # (rejected: NFI_TILE_AB 2's VOP3 v_fma_f32 vD, vA, vB, vD under gpr_idx(SRC2,DST) gave wrong
            #  d planes and a faulting launch on MI355X — DESIGN.md §3)
            if not ok_add:
                bad.append((kernel, j, f'unexpected instruction in an indexed region ({mode}): {t}'))
    return bad


LDS_RET = ('ds_read', 'ds_load', 'ds_bpermute', 'ds_permute', 'ds_swizzle', 'ds_consume', 'ds_append')


SMEM_RET = ('s_load', 's_buffer_load')


def lds_return_in_region(path: str, depth: int = 600, smem: bool = False):
    """Rule 4: for every s_set_gpr_idx_on, walk back (along the fall-through path and, at a loop
    header, from each backward branch to it) to the wait that covers it: an LDS load issued after the
    last s_waitcnt lgkmcnt(0) — or among the N most recent lgkm instructions before an lgkmcnt(N) —
    may still return its data while the region's index mode is on.  Returns (kernel, line, load)."""
    lines = open(path).read().splitlines()
    out = []
    # kernel bodies: (name, [(line no, kind, text)])
    bodies, cur = [], None
    for i, ln in enumerate(lines):
        if re.match(r'^_Z\S+:', ln):
            cur = (ln.split(':')[0], [])
            bodies.append(cur)
            continue
        if cur is None:
            continue
        if ln.startswith('.Lfunc_end'):
            cur = None
            continue
        m = re.match(r'^(\.LBB\w+):', ln)
        if m:
            cur[1].append((i + 1, 'label', m.group(1)))
            continue
        t = ln.split(';')[0].strip()
        if t and not t.startswith('.') and ln.startswith('\t'):
            cur[1].append((i + 1, 'op', t))
    for kernel, ins in bodies:
        if not any(k == 'op' and t.startswith('s_set_gpr_idx_on') for _, k, t in ins):
            continue
        labels = {t: j for j, (_, k, t) in enumerate(ins) if k == 'label'}
        back = {}
        for j, (_, k, t) in enumerate(ins):
            if k == 'op':
                m = re.match(r's_(?:cbranch_\w+|branch)\s+(\.LBB\w+)', t)
                if m and m.group(1) in labels and labels[m.group(1)] < j:
                    back.setdefault(labels[m.group(1)], []).append(j)

        def lgkm(t):
            return t.startswith(('ds_', 's_load', 's_buffer_load'))

        for j, (lno, k, t) in enumerate(ins):
            if k != 'op' or not t.startswith('s_set_gpr_idx_on'):
                continue
            stack, seen, hit = [(j - 1, 0)], set(), None
            while stack and hit is None:
                p, n = stack.pop()
                while p >= 0 and n < depth and hit is None:
                    _, kk, tt = ins[p]
                    if kk == 'label':
                        for b in back.get(p, []):
                            if b not in seen:
                                seen.add(b)
                                stack.append((b, n))
                        p -= 1
                        continue
                    if tt.startswith('s_waitcnt'):
                        mm = re.search(r'lgkmcnt\((\d+)\)', tt)
                        if mm:
                            left, q = int(mm.group(1)), p - 1
                            if left and smem:   # scalar loads return out of order: only lgkmcnt(0) completes them
                                n += 1
                                p -= 1
                                continue
                            while left > 0 and q >= 0:
                                if ins[q][1] == 'op' and lgkm(ins[q][2]):
                                    left -= 1
                                    if ins[q][2].startswith(LDS_RET):
                                        hit = ins[q]
                                q -= 1
                            break
                    if tt.startswith(LDS_RET) or (smem and tt.startswith(SMEM_RET)):
                        hit = ins[p]
                    n += 1
                    p -= 1
            if hit:
                what = 'scalar' if hit[2].startswith(SMEM_RET) else 'LDS'
                out.append((kernel, lno, f'{what} load possibly in flight at the region: line {hit[0]} {hit[2]}'))
    return out


def valu_sgpr_near_region(path: str, window: int = 30):
    """Rule 5: no VALU instruction writing an SGPR from a VGPR lane (v_readfirstlane / v_readlane)
    within `window` instructions before an s_set_gpr_idx_on, along the fall-through path and loop back
    edges — an index SGPR made that way gave wrong register images in a region train (probe patterns
    16-18).  Returns (kernel, line, message)."""
    lines = open(path).read().splitlines()
    out, bodies, cur = [], [], None
    for i, ln in enumerate(lines):
        if re.match(r'^_Z\S+:', ln):
            cur = (ln.split(':')[0], [])
            bodies.append(cur)
            continue
        if cur is None:
            continue
        if ln.startswith('.Lfunc_end'):
            cur = None
            continue
        m = re.match(r'^(\.LBB\w+):', ln)
        if m:
            cur[1].append((i + 1, 'label', m.group(1)))
            continue
        t = ln.split(';')[0].strip()
        if t and not t.startswith('.') and ln.startswith('\t'):
            cur[1].append((i + 1, 'op', t))
    for kernel, ins in bodies:
        labels = {t: j for j, (_, k, t) in enumerate(ins) if k == 'label'}
        back = {}
        for j, (_, k, t) in enumerate(ins):
            if k == 'op':
                m = re.match(r's_(?:cbranch_\w+|branch)\s+(\.LBB\w+)', t)
                if m and m.group(1) in labels and labels[m.group(1)] < j:
                    back.setdefault(labels[m.group(1)], []).append(j)
        for j, (lno, k, t) in enumerate(ins):
            if k != 'op' or not t.startswith('s_set_gpr_idx_on'):
                continue
            stack, seen, hit = [(j - 1, 0)], set(), None
            while stack and hit is None:
                p, n = stack.pop()
                while p >= 0 and n < window:
                    _, kk, tt = ins[p]
                    if kk == 'label':
                        for b in back.get(p, []):
                            if b not in seen:
                                seen.add(b)
                                stack.append((b, n))
                        p -= 1
                        continue
                    if tt.startswith(('v_readfirstlane', 'v_readlane')):
                        hit = ins[p]
                        break
                    n += 1
                    p -= 1
            if hit:
                out.append((kernel, lno, f'VALU-written SGPR {window} instructions or fewer before the region: '
                                         f'line {hit[0]} {hit[2]}'))
    return out


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
        g = lint_gpr_idx(out) + lds_return_in_region(out, smem=True) + valu_sgpr_near_region(out)
        nreg = sum(1 for ln in open(out) if 's_set_gpr_idx_on' in ln)
        print(f'{os.path.basename(s)}: {nreg} M0-indexed regions, {len(g)} violations')
        for k, ln, msg in g:
            print(f'  {k[:70]}  line {ln}: {msg}')
        total += g
    print('isa lint:', 'FAIL' if total else 'ok')
    return 1 if total else 0


if __name__ == '__main__':
    sys.exit(main())
