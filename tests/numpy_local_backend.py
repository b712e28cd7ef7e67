"""TEST INFRASTRUCTURE: a numpy implementation of the libvgposp local-greedy calls
(vgposp_local_score / _argmax / _pick semantics, through the oracle's local deltas) so that the
multi-rank orchestration of vgposp_amd.local_placement runs with gloo on CPU.  Never used by the
product."""
import numpy as np
import torch

from oracle import local_placement as lp
from vgposp_amd.local_placement import plane_slabs


class NumpyLocalBackend:
    def __init__(self, X, shape, kmax, cutoff, beta, rank=0, world=1, **kw):
        self.X = np.asarray(X, dtype=np.float64)
        self.shape = tuple(shape)
        self.n = int(np.prod(shape))
        self.kmax, self.cutoff, self.beta, self.kw = kmax, cutoff, beta, kw
        self.c0, self.c1 = plane_slabs(shape, world)[rank]
        self.selected = np.zeros(self.n, dtype=bool)
        self.picks = torch.full((kmax,), -1, dtype=torch.int64)
        self.pick_delta = torch.zeros(kmax, dtype=torch.float64)
        self.cache = np.zeros(self.c1 - self.c0)
        self.key = torch.zeros(2, dtype=torch.int64)

    def reset(self):
        self.selected[:] = False
        self.picks.fill_(-1)

    def _deltas(self, cand):
        return lp.local_deltas(self.X, self.shape, cand, self.selected, self.beta, **self.kw)

    def score_all(self):
        self.cache[:] = self._deltas(np.arange(self.c0, self.c1))

    def window(self, rnd):
        w = lp.window(int(self.picks[rnd]), self.shape, self.cutoff)
        w = w[(w >= self.c0) & (w < self.c1)]
        if len(w):
            self.cache[w - self.c0] = self._deltas(w)

    def argmax(self, rnd):
        c = np.where(self.selected[self.c0:self.c1], -np.inf, self.cache)
        i = int(np.argmax(c)) if len(c) else -1
        v = float(self.cache[i]) if i >= 0 else 0.0
        self.key[0] = int(np.float64(v).view(np.int64))
        self.key[1] = self.c0 + i if i >= 0 else -1
        return self.key

    def pick(self, keys, nkeys, rnd, window=True):
        best_v, best_i = 0.0, -1
        for q in range(nkeys):
            v = float(np.int64(keys[2 * q]).view(np.float64))
            i = int(keys[2 * q + 1])
            if i < 0:
                continue
            if best_i < 0 or v > best_v or (v == best_v and i < best_i):
                best_v, best_i = v, i
        self.picks[rnd] = best_i
        self.pick_delta[rnd] = best_v
        self.selected[best_i] = True
        if self.c0 <= best_i < self.c1:
            self.cache[best_i - self.c0] = 0.0
        if window:
            self.window(rnd)

    def local_cache(self):
        return torch.as_tensor(self.cache)
