"""The stage-2 pipeline's lag-3 rule preserves the reference's serial order.

Task t of sweep i may start once task t+3 of sweep i-1 is done
(brd_stage2.hip, k_band2bd_pipe).  This holds iff every pair of overlapping
windows (i, t), (i', t') with i < i' satisfies t <= t' + 3 (i' - i).  The
windows are enumerated exactly as the reference's brd_p2 builds them
(svd_parallel.h:648-688), including clipped and empty ones.
"""
import pytest


def windows(m, n, b, sigma=False):
    bs = b + 1
    W = {}
    for i in range(n - 1):
        tl = (i, min(i + bs, m), i + 1, min(i + bs, n))
        tasks = [tl]
        tl = (i + 1, min(i + bs, m), i + 1, min(i + 2 * bs - 1, n))
        tasks.append(tl)
        nbtx = (n - tl[3]) // (bs - 1) + (1 if sigma else 0)
        for _ in range(nbtx + 1):
            end_i = min(tl[1] + bs - 1, m)
            sj = min(tl[2] + bs - 1, n)
            ej3 = min(tl[3] + bs - 1, n)
            tr = (tl[0], end_i, sj, tl[3])
            tl = (tl[1], end_i, sj, ej3)
            tasks += [tr, tl]
        W[i] = [t if (t[3] > t[2] and t[1] > t[0]) else None for t in tasks]
    return W


def _overlap(a, b):
    return a[0] < b[1] and b[0] < a[1] and a[2] < b[3] and b[2] < a[3]


def worst_slack(n, b, lag, sigma=False):
    W = windows(n, n, b, sigma)
    worst = -10 ** 9
    for i in W:
        for ip in range(i + 1, min(n - 1, i + 2 * b + 4)):
            for t, wa in enumerate(W[i]):
                if wa is None:
                    continue
                for tp, wb in enumerate(W[ip]):
                    if wb is not None and _overlap(wa, wb):
                        worst = max(worst, t - tp - lag * (ip - i))
    return worst


@pytest.mark.parametrize("sigma", [False, True])
@pytest.mark.parametrize("n,b", [(64, 4), (100, 4), (130, 8), (128, 32), (257, 32), (300, 16), (50, 2), (40, 1)])
def test_lag3_preserves_serial_order(n, b, sigma):
    assert worst_slack(n, b, 3, sigma) <= 0


@pytest.mark.parametrize("n,b", [(64, 4), (128, 32)])
def test_lag2_is_not_enough(n, b):
    assert worst_slack(n, b, 2) > 0


@pytest.mark.parametrize("sigma", [False, True])
def test_windows_fit_kernel_limits(sigma):
    """Right windows <= 2b x b, left windows <= b x 2b (one row/column per lane)."""
    for n, b in [(257, 32), (100, 4), (64, 1)]:
        for i, tasks in windows(n, n, b, sigma).items():
            for t, w in enumerate(tasks):
                if w is None:
                    continue
                rows, cols = w[1] - w[0], w[3] - w[2]
                if t % 2 == 0:
                    assert rows <= max(2 * b, b + 1) and cols <= b
                else:
                    assert rows <= b and cols <= 2 * b


def ring_min_rows(b, S):
    """Mirror of brd_stage2.hip ring_min_rows()."""
    return ((3 * (S - 1)) // 2 + 2) * b + S + 8


def exact_ring_need(n, b, S, sigma=False):
    """Rows the LDS ring must hold so the trailing sweep of a bundle can always
    progress: from the trailing sweep's next window top to the bottom of the
    leading sweep's window 3(S-1) tasks ahead (its predecessors' bottoms are
    at most S-1 rows lower)."""
    W = windows(n, n, b, sigma)
    worst = 0
    for i0 in range(0, n - S):
        lead, trail = W[i0], W[i0 + S - 1]
        for tau, w in enumerate(trail):
            if w is None:
                continue
            hi = min(tau + 3 * (S - 1), len(lead) - 1)
            bots = [x[1] for x in lead[:hi + 1] if x is not None] + [w[1]]
            worst = max(worst, max(bots) + (S - 1) - w[0])
    return worst


@pytest.mark.parametrize("n,b,S", [(300, 32, 1), (300, 32, 2), (300, 32, 3), (300, 32, 4), (300, 32, 7), (200, 4, 15),
                                   (120, 8, 5), (400, 16, 6), (257, 32, 5), (150, 2, 9)])
def test_ring_size_formula_is_sufficient(n, b, S):
    assert ring_min_rows(b, S) >= exact_ring_need(n, b, S)
    assert ring_min_rows(b, S) >= exact_ring_need(n, b, S, sigma=True)


def corner_rule_violations(n, b, sigma=False):
    """A finer schedule than lag 3 (measured and not kept, DESIGN.md stage 2
    round 2): window t of sweep i+1 starts once sweep i has finished window
    t+2, and only its bottom-right corner's row (right window) or column (left
    window) waits for window t+3.
    Transitively, when window t of sweep i+d starts, sweep i has finished
    windows up to t+3d-1, and when its corner part runs, up to t+3d.  Valid iff
    every overlap with a later window of an earlier sweep is exactly that
    corner element, at distance d = 1, and the corner is not in the window's
    source row / column.  Returns the violating pairs."""
    W = windows(n, n, b, sigma)
    bad = []
    for i in W:
        for d in range(1, 2 * b + 6):
            ip = i + d
            if ip not in W:
                break
            for tp, wb in enumerate(W[ip]):
                if wb is None:
                    continue
                right = tp % 2 == 0
                corner = (wb[1] - 1, wb[1], wb[3] - 1, wb[3])
                for t, wa in enumerate(W[i]):
                    if wa is None or t < tp + 3 * d or not _overlap(wa, wb):
                        continue
                    inter = (max(wa[0], wb[0]), min(wa[1], wb[1]), max(wa[2], wb[2]), min(wa[3], wb[3]))
                    src_ok = (wb[1] - 1 > wb[0]) if right else (wb[3] - 1 > wb[2])
                    if not (d == 1 and t == tp + 3 and inter == corner and src_ok):
                        bad.append((i, t, ip, tp))
    return bad


@pytest.mark.parametrize("sigma", [False, True])
@pytest.mark.parametrize("n,b", [(300, 32), (257, 32), (130, 8), (100, 4), (50, 2), (40, 1), (333, 16)])
def test_lag2_corner_rule_preserves_serial_order(n, b, sigma):
    assert corner_rule_violations(n, b, sigma) == []
