"""Communication observability: per-role collective time and the fraction hidden under compute.

The reference reports one wall time per method (train_ffns.py:378-382); nothing says how long its
collectives took or whether they overlapped anything.  ``CommObserver`` answers both from HIP events,
for either communicator backend (torch ProcessGroupNCCL or the native RCCL layer):

* every collective issued through ``parallel.comm`` records an *issue* event on the caller's stream, and an
  *end* event on a per-role observer stream that waits on the collective's completion (``work.wait()``
  under that stream) -- so the end timestamp is the collective's completion, whatever stream ran it;
* the native RCCL layer (``parallel/rccl.py``) records the two events on its communicator stream itself,
  after the input wait and after the kernel: its intervals are execution intervals, as in a kernel trace
  (torch ProcessGroupNCCL keeps its stream private, so there the interval runs from issue to completion
  and carries the launch / event latency: ~20-30 us per collective);
* a collective queued behind an earlier one of its role cannot start before that one ends, so its start is
  ``max(issue, previous end of the role)`` (one communicator = one stream per role);
* a collective that moves no data (in place on a size-1 communicator: ``force_comm`` at N=1) launches no
  kernel; it is counted but kept out of the intervals, as a kernel trace of the same run has nothing for it;
* every native GEMM records events around its launch on the compute stream (``ops.gemm`` calls
  ``gemm_begin`` / ``gemm_end``); the start event fires when the GEMM can start (after any stream wait).

``summary()`` (after a device synchronize) reports per role the collective time per step, the union of
all collective intervals, how much of it intersects the union of GEMM intervals (``hidden``), and
``overlap_frac = hidden / union``.  Observation costs a few events per collective / GEMM, so drivers run
it on extra steps after the timed ones (bench.py), never inside the timed region.
"""
from __future__ import annotations

import torch

_OBS: "CommObserver | None" = None


def active() -> "CommObserver | None":
    return _OBS


def _union(iv: list[tuple[float, float]]) -> list[tuple[float, float]]:
    out: list[list[float]] = []
    for s, e in sorted(iv):
        if e <= s:
            continue
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return [(s, e) for s, e in out]


def _length(iv) -> float:
    return sum(e - s for s, e in iv)


def _intersect(a, b) -> float:
    i = j = 0
    tot = 0.0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if e > s:
            tot += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


class CommObserver:
    def __init__(self, device: torch.device, roles: dict | None = None):
        self.device = torch.device(device)
        self.roles = {id(g): r for r, g in (roles or {}).items() if g is not None}
        self.obs_streams: dict[str, torch.cuda.Stream] = {}
        self.colls: list[tuple[str, torch.cuda.Event, torch.cuda.Event]] = []
        self.n_noop = 0  # collectives that moved no data (counted, no interval)
        self.gemms: list[tuple[torch.cuda.Event, torch.cuda.Event]] = []
        self._open: torch.cuda.Event | None = None
        self.t0: torch.cuda.Event | None = None
        self.steps = 0

    # -- lifecycle -------------------------------------------------------------------------------------
    def __enter__(self):
        global _OBS
        # observer streams are created (and their first command retired) up front: a stream's first command runs
        # late (measured: ~0.3 ms), which would stretch the first collective of each role
        for role in set(self.roles.values()) | {"other"}:
            st = self.obs_streams.setdefault(role, torch.cuda.Stream(device=self.device))
            torch.cuda.Event(enable_timing=True).record(st)
        torch.cuda.synchronize(self.device)
        self.t0 = torch.cuda.Event(enable_timing=True)
        self.t0.record(torch.cuda.current_stream(self.device))
        _OBS = self
        return self

    def __exit__(self, *exc):
        global _OBS
        _OBS = None
        return False

    # -- hooks -----------------------------------------------------------------------------------------
    def role_of(self, group) -> str:
        return self.roles.get(id(group), "other")

    def issue(self) -> torch.cuda.Event:
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(self.device))
        return ev

    def issued(self, group, ev_issue: torch.cuda.Event, work, moves: bool = True) -> None:
        if not moves:
            self.n_noop += 1
            return
        role = self.role_of(group)
        span = getattr(work, "span", None)
        if span is not None:  # native communicator: timing events on its own stream around the kernel
            self.colls.append((role, span[0], span[1]))
            return
        st = self.obs_streams.get(role)
        if st is None:
            st = self.obs_streams[role] = torch.cuda.Stream(device=self.device)
        st.wait_event(ev_issue)  # the observer stream may not run ahead of the issue point
        with torch.cuda.stream(st):
            work.wait()  # observer stream waits on the collective's completion (no host block)
            end = torch.cuda.Event(enable_timing=True)
            end.record(st)
        self.colls.append((role, ev_issue, end))

    def gemm_begin(self) -> None:
        self._open = torch.cuda.Event(enable_timing=True)
        self._open.record(torch.cuda.current_stream(self.device))

    def gemm_end(self) -> None:
        if self._open is None:
            return
        end = torch.cuda.Event(enable_timing=True)
        end.record(torch.cuda.current_stream(self.device))
        self.gemms.append((self._open, end))
        self._open = None

    # -- report ----------------------------------------------------------------------------------------
    def intervals(self) -> tuple[dict, list]:
        """Raw (ms since observation start) collective intervals per role and GEMM intervals (diagnostics)."""
        torch.cuda.synchronize(self.device)
        t = lambda ev: self.t0.elapsed_time(ev)  # noqa: E731  (ms since observation start)
        per_role: dict[str, list[tuple[float, float]]] = {}
        last_end: dict[str, float] = {}
        for role, ev_i, ev_e in self.colls:
            s, e = t(ev_i), t(ev_e)
            s = max(s, last_end.get(role, s))  # queued behind the role's previous collective
            last_end[role] = max(e, last_end.get(role, e))
            per_role.setdefault(role, []).append((s, e))
        return per_role, [(t(a), t(b)) for a, b in self.gemms]

    def summary(self, steps: int) -> dict:
        per_role, gemms = self.intervals()
        gem = _union(gemms)
        allc = _union([iv for ivs in per_role.values() for iv in ivs])
        union_ms, hidden = _length(allc), _intersect(allc, gem)
        steps = max(1, steps)
        return {
            "comm_ms": round(union_ms / steps, 3),
            "comm_ms_by_role": {r: round(_length(_union(iv)) / steps, 3) for r, iv in sorted(per_role.items())},
            "collectives_per_step": round((len(self.colls) + self.n_noop) / steps, 1),
            "noop_collectives_per_step": round(self.n_noop / steps, 1),
            "comm_hidden_ms": round(hidden / steps, 3),
            "comm_exposed_ms": round((union_ms - hidden) / steps, 3),
            "overlap_frac": round(hidden / union_ms, 4) if union_ms > 0 else None,
            "gemm_busy_ms": round(_length(gem) / steps, 3),
        }
