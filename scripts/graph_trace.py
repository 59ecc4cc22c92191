"""Summarise the eager vs graph-replayed kernel traces of scripts/graph_trace.sh: for the timed
inversion steps (the last 10 'nfi::tile_kernel' launches mark one step each), per step: kernels,
summed kernel time (busy, both streams), span, the busy time of the union of kernel intervals,
idle time between kernels (span - union), and the median / p90 gap between consecutive kernels."""
import csv
import glob
import statistics
import sys


def load(d):
    f = glob.glob(f'{d}/**/*kernel_trace.csv', recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    ks = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'], r.get('Queue_Id', r.get('Stream_Id', '')))
          for r in rows]
    ks.sort()
    return ks


def steps(ks, n=10):
    marks = [i for i, k in enumerate(ks) if 'tile_kernel' in k[2]]
    # the inversion leg runs after the render bench: its steps are the last n + a few tile launches;
    # a step = from the kernel after one tile_kernel... use the spacing between consecutive marks
    marks = marks[-(n + 1):]
    out = []
    for a, b in zip(marks, marks[1:]):
        seg = ks[a + 1:b + 1]
        busy = sum(e - s for s, e, _, _ in seg)
        span = seg[-1][1] - seg[0][0]
        union, cur_s, cur_e = 0, None, None
        for s, e, _, _ in seg:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    union += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        union += cur_e - cur_s
        gaps = [max(0, seg[i + 1][0] - seg[i][1]) for i in range(len(seg) - 1)]
        queues = len({q for _, _, _, q in seg})
        out.append(dict(kernels=len(seg), busy=busy / 1e6, span=span / 1e6, union=union / 1e6,
                        idle=(span - union) / 1e6, gap_med=statistics.median(gaps) / 1e3,
                        gap_p90=sorted(gaps)[int(0.9 * len(gaps))] / 1e3, queues=queues))
    return out


def main():
    for d in sys.argv[1:]:
        st = steps(load(d))
        med = {k: statistics.median([s[k] for s in st]) for k in st[0]}
        print(f'{d}: per step (median of {len(st)}): kernels {med["kernels"]:.0f}, kernel time {med["busy"]:.3f} ms, '
              f'span {med["span"]:.3f} ms, busy union {med["union"]:.3f} ms, idle {med["idle"]:.3f} ms, '
              f'gap median {med["gap_med"]:.2f} us, p90 {med["gap_p90"]:.2f} us, queues {med["queues"]:.0f}')


if __name__ == '__main__':
    main()
