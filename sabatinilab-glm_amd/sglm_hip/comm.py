"""Row-sharded solves over a process group (the rows of one CV grid split
over the ranks).

The reference partitions the CV grid by fold onto worker threads (backend/sglm_cv.py:162-170);
on one MI355X node the fits of one grid are latency-bound on a GPU's share, so the grid is
also split by ROWS: every rank holds one contiguous slab of the design rows (its own bit
planes, masks and responses) and runs the SAME Newton iterations over ALL fits.  Every
quantity that is a sum over rows -- Grams XᵀWX, gradients Xᵀr, trial losses, score sums, mask
statistics -- is all-reduced (RCCL over xGMI), every maximum over rows (predictor drift, the
λ-neighbour / alias pair distances) max-reduced; all ranks then hold bitwise identical values
(a ring / tree all-reduce computes each element once and broadcasts it), so their host
decisions -- step lengths, stopping, Hessian reuse -- agree without further exchange.  The
new factorisations of an iteration are dealt round-robin over the ranks; a rank solves the
fits whose factor it holds and the Newton directions are combined by one sum in which every
other rank contributes zeros.

``RowComm`` is the process-group implementation.  ``SimComm`` stands in for it in one-GPU
timing simulations (tools/rank_sim.py --mode rows): the collectives' results and the other
ranks' directions are replayed from a recording of the unsharded grid, so a rank's slab
follows the row-sharded trajectory while only its own work runs."""
from __future__ import annotations

import numpy as np


def row_slab(n: int, rank: int, world: int, align: int = 64):
    """Rows [start, stop) of ``rank``'s slab of ``n`` rows: near-equal contiguous runs whose
    boundaries are multiples of ``align`` (compacted bit-plane blocks stay whole; single rows
    when n < align * world)."""
    if world <= 1:
        return 0, int(n)
    if n < world:
        raise ValueError(f"{n} rows cannot be split over {world} ranks")
    if n < align * world:
        align = 1
    cuts = [min(int(n), int(round(n * q / world / align)) * align) for q in range(world + 1)]
    cuts[-1] = int(n)
    return cuts[rank], cuts[rank + 1]


class RowComm:
    """Collectives of a row-sharded solve over an initialised torch.distributed group."""
    distribute = True                    # factorisations dealt over the ranks

    def __init__(self, dist):
        self.dist = dist
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.calls = 0
        self.bytes = 0

    def _note(self, t):
        self.calls += 1
        self.bytes += t.numel() * t.element_size()

    def sum_(self, t):
        """In-place sum over ranks (t contiguous, on this rank's device)."""
        self._note(t)
        self.dist.all_reduce(t)

    def max_(self, t):
        self._note(t)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)

    def min_(self, t):
        self._note(t)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN)

    def directions_(self, delta, owned_d=None):
        """Combine the Newton directions: each fit's row is nonzero on its owner only.
        ``owned_d``: device uint8 flags of the rows this rank solved (SimComm's replay)."""
        self.sum_(delta)

    def sum_owned_(self, t):
        """Sum of values each of which only its owner rank holds (others contribute 0)."""
        self.sum_(t)

    def owners(self, nform: int, rot: int) -> np.ndarray:
        """Owner rank of each of an iteration's ``nform`` new factorisations (round-robin,
        rotated by ``rot`` so that consecutive iterations start on different ranks)."""
        return (np.arange(nform, dtype=np.int64) + rot) % self.world


class SimComm(RowComm):
    """One rank's share of a row-sharded solve, timed on one GPU without a process group.

    ``SimComm.recorder()`` runs the UNSHARDED grid (full design) and keeps, in call order, the
    value every collective of a row-sharded run would return -- the global sums and maxima --
    and every Newton iteration's directions; its factorisations all run locally.
    ``recorder.replay(rank, world)`` then runs that rank's slab: each collective overwrites the
    slab's partial with the recorded global value (a device copy instead of the all-reduce),
    the rank factors only its round-robin share and takes the other fits' directions from the
    recording.  The replay thus follows the row-sharded run's trajectory (up to the summation
    order of the global sums) and times the slab's own work; the collectives are not timed."""

    def __init__(self, rank: int = 0, world: int = 1, record: bool = True, tape=None):
        self.rank, self.world = int(rank), int(world)
        self.record = bool(record)
        self.distribute = not self.record
        self.tape = [] if tape is None else tape
        self._k = 0
        self.calls = 0
        self.bytes = 0

    @classmethod
    def recorder(cls):
        return cls(0, 1, record=True)

    def replay(self, rank: int, world: int):
        return SimComm(rank, world, record=False, tape=self.tape)

    def _value_(self, t):
        self._note(t)
        if self.record:
            self.tape.append(t.clone())
            return
        rec = self.tape[self._k]
        self._k += 1
        if rec.shape != t.shape or rec.dtype != t.dtype:
            raise RuntimeError(f"SimComm replay out of step: recorded {tuple(rec.shape)} "
                               f"{rec.dtype}, got {tuple(t.shape)} {t.dtype}")
        t.copy_(rec)

    sum_ = max_ = min_ = _value_

    def sum_owned_(self, t):
        """Per-owner values (dropped-pivot counts) stay local in a simulation."""

    def directions_(self, delta, owned_d=None):
        self._note(delta)
        if self.record:
            self.tape.append(delta.clone())
            return
        import torch
        rec = self.tape[self._k]
        self._k += 1
        delta.copy_(torch.where(owned_d[: delta.shape[0], None].bool(), delta, rec))
