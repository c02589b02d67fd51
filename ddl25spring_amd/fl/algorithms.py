"""Horizontal FL algorithms on the client-batched engine, one MI355X = a group of client slots.

FedAvg (McMahan et al. 2017) and FedSGD with the reference's exact round protocol
(hfl_complete.py:220-229, 260-312, 336-390):
  * ``K = max(1, round(C * N))`` clients sampled per round with ``numpy.default_rng(seed).choice(N,
    K, replace=False)`` — every rank draws the same numbers, no communication needed;
  * client ``c`` in round ``r`` shuffles its data with seed ``seed + c + 1 + r * K``;
  * weights ``n_k / sum(n_chosen)``; ``message_count = 2 * (r + 1) * K``.
Placement: chosen client ``i`` of a round runs on rank ``i % W``, slot ``i // W``; every rank holds
the (device-resident) training set, the server state ``w_global`` is replicated and updated
identically on every rank after the all-reduce, so there is no separate parameter-server process.
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from ..ops import functional as Fn
from ..runtime import dist as rdist
from ..utils.metrics import PhaseTimer
from .aggregate import MeanAggregator, make_aggregator
from .local import LocalTrainer
from .result import RunResult


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


class FederatedBase:
    algorithm = "Fed"

    def __init__(self, model_fn, train_data, client_indices, *, lr: float, batch_size: int = -1,
                 local_epochs: int = 1, client_fraction: float = 1.0, seed: int = 0, test_data=None,
                 aggregator="mean", attack=None, ctx=None, momentum: float = 0.0,
                 weight_decay: float = 0.0, planner: str = "native", use_graph=None,
                 init_fn=None, eval_every: int = 1, eval_limit: int | None = None, name=None,
                 agg_kwargs=None, dropout: float = 0.0, stragglers: float = 0.0,
                 straggler_slowdown: float = 4.0, deadline: float | None = None):
        self.ctx = ctx or rdist.context()
        self.dev = self.ctx.device
        self.data = train_data
        self.test_data = test_data
        self.client_indices = [np.asarray(c, dtype=np.int64) for c in client_indices]
        self.N = len(self.client_indices)
        self.C = client_fraction
        self.K = max(1, round(client_fraction * self.N))
        self.W = self.ctx.world
        self.slots = math.ceil(self.K / self.W)
        self.lr, self.B, self.E, self.seed = lr, batch_size, local_epochs, seed
        self.rng = np.random.default_rng(seed)
        self.counts = [len(c) for c in self.client_indices]
        self.net = model_fn(groups=self.slots).to(self.dev, seed=seed)
        if init_fn is not None:
            init_fn(self.net)
        self.data.set_input_spec(self.net.input_spec)
        if self.test_data is not None:
            self.test_data.set_input_spec(self.net.input_spec)
        st = self.net.store
        self.w_global = st.data[0].clone()
        self.b_global = st.buffers[0].clone()
        self.aggregator = aggregator if not isinstance(aggregator, str) else \
            make_aggregator(aggregator, **(agg_kwargs or {}))
        self.mean = MeanAggregator()
        self.attack = attack
        self.momentum, self.weight_decay = momentum, weight_decay
        self.planner, self.use_graph = planner, use_graph
        self.eval_every, self.eval_limit = eval_every, eval_limit
        self.name = name or self.algorithm
        self.round_idx = 0
        # [NS] client unavailability: each sampled client independently fails to report with
        # probability ``dropout`` (own RNG stream, so the client-sampling sequence is unchanged)
        self.dropout = dropout
        self.fail_rng = np.random.default_rng([seed, 0xD20])
        self.dropped: list[list[int]] = []
        # [NS] stragglers: each sampled client is independently slow with probability
        # ``stragglers`` (its local round takes ``straggler_slowdown`` x the nominal time of its
        # shard, n_k * E samples at unit speed). With a ``deadline`` (in nominal times of the mean
        # shard) the server aggregates only the clients that report in time, the synchronous-FL
        # policy of dropping stragglers; ``sim_time`` records each round's simulated duration
        # (slowest reporting client), the reference's "parallel wall time = max over clients"
        # (hfl_complete.py:294,296) under heterogeneous client speed.
        self.stragglers, self.slowdown, self.deadline = stragglers, straggler_slowdown, deadline
        self.strag_rng = np.random.default_rng([seed, 0x57A6])
        self.straggled: list[list[int]] = []
        self.sim_time: list[float] = []
        self.timer = PhaseTimer(self.dev)  # download / local_train / aggregate (HIP events + roctx)
        # sync_rounds=False: FedAvg rounds run without any host <-> device synchronisation (no
        # per-round wall time; round() returns dt = 0 and this rank's sample count), so the host
        # samples, plans and enqueues round r+1 while the GPU still executes round r. For
        # throughput runs (bench.py); run() keeps the reference's per-round timing.
        self.sync_rounds = True
        self._coeff_cache: dict = {}

    def _sample(self):
        chosen = self.rng.choice(self.N, self.K, replace=False)
        if self.dropout > 0:
            alive = self.fail_rng.random(len(chosen)) >= self.dropout
            self.dropped.append([int(c) for c in chosen[~alive]])
            chosen = chosen[alive]
        if self.stragglers > 0:
            slow = self.strag_rng.random(len(chosen)) < self.stragglers
            mean_n = float(np.mean(self.counts))
            t = np.array([self.counts[int(c)] / mean_n for c in chosen]) * \
                np.where(slow, self.slowdown, 1.0)
            late = t > self.deadline if self.deadline is not None else np.zeros(len(chosen), bool)
            self.straggled.append([int(c) for c in chosen[late]])
            self.sim_time.append(float(t[~late].max()) if (~late).any() else 0.0)
            chosen = chosen[~late]
        return chosen

    # ------------------------------------------------------------------ checkpoint / resume
    def state_dict(self) -> dict:
        """Everything needed to continue bit-identically: server model, round counter, RNG streams
        (loader seeds derive from seed/round/client, so they need no state)."""
        sd = {"w_global": self.w_global.detach().cpu().clone(),
              "b_global": self.b_global.detach().cpu().clone(),
              "round_idx": self.round_idx, "rng": self.rng.bit_generator.state,
              "fail_rng": self.fail_rng.bit_generator.state, "dropped": self.dropped,
              "strag_rng": self.strag_rng.bit_generator.state, "straggled": self.straggled,
              "sim_time": self.sim_time,
              "algorithm": self.algorithm, "N": self.N, "K": self.K, "seed": self.seed,
              "param_layout": self.net.store.param_layout()}
        for name in ("g_global",):
            if hasattr(self, name):
                sd[name] = getattr(self, name).detach().cpu().clone()
        if self.attack is not None:
            sd["attack"] = self.attack.state_dict()
        return sd

    def load_state_dict(self, sd: dict) -> None:
        if (sd["algorithm"], sd["N"], sd["K"]) != (self.algorithm, self.N, self.K):
            raise ValueError("checkpoint is for a different federation "
                             f"{(sd['algorithm'], sd['N'], sd['K'])}")
        # flat rows are remapped by parameter name when the writer used another layout
        st = self.net.store
        src = sd.get("param_layout") or st.param_layout()
        fix = (lambda t: t) if [list(x) for x in src] == st.param_layout() else \
            (lambda t: st.remap_flat(t, src))
        self.w_global.copy_(fix(sd["w_global"]).to(self.dev))
        self.b_global.copy_(sd["b_global"].to(self.dev))
        if "g_global" in sd and hasattr(self, "g_global"):
            self.g_global.copy_(fix(sd["g_global"]).to(self.dev))
        self.round_idx = int(sd["round_idx"])
        self.rng.bit_generator.state = sd["rng"]
        self.fail_rng.bit_generator.state = sd["fail_rng"]
        self.dropped = [list(d) for d in sd["dropped"]]
        if "strag_rng" in sd:
            self.strag_rng.bit_generator.state = sd["strag_rng"]
            self.straggled = [list(d) for d in sd["straggled"]]
            self.sim_time = list(sd["sim_time"])
        if self.attack is not None and "attack" in sd:
            self.attack.load_state_dict(sd["attack"])

    # ------------------------------------------------------------------ helpers
    def _assign(self, chosen):
        mine = [int(c) for c in chosen[self.ctx.rank::self.W]]
        counts = [len(chosen[i::self.W]) for i in range(self.W)]
        return mine, counts

    def _row_keys(self, counts):
        """Each rank-major client row's position in the round's `chosen` order (round-robin
        assignment above): the robust rules break exact ties by it, so a run gives the same
        aggregate on one GPU and on W."""
        return [l * self.W + w for w in range(self.W) for l in range(counts[w])]

    def _download(self, G):
        st = self.net.store
        if G:
            Fn.broadcast_rows(self.w_global, st.data[:G], None if st.shadow16 is None else st.shadow16[:G])
            Fn.broadcast_rows(self.b_global, st.buffers[:G])
            st._shadow_version = st.data._version

    def _mean_buffers(self, G, coeffs):
        st = self.net.store
        self.mean(self.ctx, st.buffers[:G], coeffs, self.b_global)

    @torch.no_grad()
    def test(self) -> float:
        """Server-model test accuracy in % (reference Server.test, hfl_complete.py:172-183)."""
        if self.test_data is None:
            return float("nan")
        st = self.net.store
        self._download(1)
        n = len(self.test_data) if self.eval_limit is None else min(self.eval_limit, len(self.test_data))
        correct = torch.zeros(1, dtype=torch.int64, device=self.dev)
        chunk = 2000
        with st.select(0, 1):
            for s in range(0, n, chunk):
                e = min(n, s + chunk)
                idx = torch.arange(s, e, dtype=torch.int32, device=self.dev).reshape(1, -1)
                x, y = self.test_data.batch(idx)
                logits, _ = self.net.forward_native(x, False)
                _, _, c = Fn.cross_entropy(logits, y, ncls=self.net.num_classes, want_grad=False,
                                           with_correct=True)
                correct += c.to(torch.int64)
        return 100.0 * correct.item() / n

    def run(self, nr_rounds: int) -> RunResult:
        res = RunResult(self.name, self.N, self.C, self.B, self.E, self.lr, self.seed)
        elapsed = 0.0
        for _ in range(nr_rounds):
            dt, samples = self.round()
            elapsed += dt
            res.wall_time.append(round(elapsed, 1))
            res.round_time.append(dt)
            res.samples.append(samples)
            res.message_count.append(2 * self.round_idx * self.K)
            res.phase_ms.append(self.timer.summary())
            if self.eval_every and self.round_idx % self.eval_every == 0:
                res.test_accuracy.append(self.test())
            else:
                res.test_accuracy.append(float("nan"))
        return res


class FedAvg(FederatedBase):
    algorithm = "FedAvg"

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.trainer = None

    def _trainer(self, mine):
        lt = None
        if self.attack is not None:
            lt = self.attack.label_transform_for(mine, self.net.num_classes)
        if self.trainer is None:
            self.trainer = LocalTrainer(self.net, self.data, self.lr, self.B, self.momentum,
                                        self.weight_decay, self.planner, self.use_graph)
            self._graph_default = self.trainer.use_graph
        self.trainer.label_transform = lt
        # a label transform is graph-captured only if it declares a graph_key (pure device ops,
        # e.g. LabelFlip); otherwise eager steps for the rounds that need one
        self.trainer.use_graph = self._graph_default and (lt is None or hasattr(lt, "graph_key"))
        return self.trainer

    def _coeffs(self, mine, total):
        """Device tensor of the n_k / n weights of my clients; cached per (clients, total), since
        building it from a host list is a blocking copy."""
        key = (tuple(mine), total)
        t = self._coeff_cache.get(key)
        if t is None:
            t = torch.tensor([self.counts[c] / total for c in mine], dtype=torch.float32, device=self.dev)
            if len(self._coeff_cache) < 256:
                self._coeff_cache[key] = t
        return t

    def round(self):
        if self.sync_rounds:
            _sync(self.dev)
        t0 = time.perf_counter()
        chosen = self._sample()
        if len(chosen) == 0:  # every sampled client dropped out: the server model stays
            self.round_idx += 1
            return self.ctx.max_scalar(time.perf_counter() - t0), 0
        mine, counts = self._assign(chosen)
        G = len(mine)
        total = float(sum(self.counts[int(c)] for c in chosen))
        r = self.round_idx
        with self.timer("download"):
            self._download(G)
        seeds = [self.seed + c + 1 + r * self.K for c in mine]
        gens = [torch.Generator().manual_seed(s) for s in seeds] if self.planner == "torch" else None
        trainer = self._trainer(mine)
        bsz = self.B
        samples = 0
        if G:
            # every slot trains in the one client-batched launch; a free rider's row is then
            # overwritten with w_global by its poison_updates (no separate code path per client)
            if bsz <= 0:  # B = infinity: full local batch
                trainer.B = max(self.counts[c] for c in mine)
            with self.timer("local_train"):
                samples = trainer.run([self.client_indices[c] for c in mine], seeds, self.E, gens)
            if self.attack is not None:  # free riders did no useful work: do not count it
                samples -= sum(self.E * self.counts[c] for c in mine if self.attack.skip_training(c))
        st = self.net.store
        if self.attack is not None and G:
            self.attack.poison_updates(st.data[:G], self.w_global, mine)
        coeffs = self._coeffs(mine, total)
        with self.timer("aggregate"):
            self._aggregate(st.data[:G], coeffs, counts)
            self._mean_buffers(G, coeffs)
        self.round_idx += 1
        if not self.sync_rounds:
            return 0.0, samples
        _sync(self.dev)
        self.ctx.check_comm()  # a peer-read all-reduce barrier timeout raises here, not silently
        dt = self.ctx.max_scalar(time.perf_counter() - t0)
        samples = int(self.ctx.sum_scalar(samples))
        return dt, samples

    def _aggregate(self, rows, coeffs, counts):
        if not getattr(self.aggregator, "needs_all", False):
            self.aggregator(self.ctx, rows, coeffs, self.w_global)
        else:
            upd = rows - self.w_global  # robust rules act on updates
            agg = self.aggregator(self.ctx, upd, counts, self.w_global.numel(), keys=self._row_keys(counts))
            self.w_global.add_(agg)


class FedSGD(FederatedBase):
    """Clients return the full-local-batch gradient at w_global; the server takes one SGD step
    with the weighted-mean gradient (reference FedSgdGradientServer, hfl_complete.py:260-312)."""
    algorithm = "FedSGDGradient"

    def __init__(self, *a, max_microbatch: int = 4096, **kw):
        kw.setdefault("batch_size", -1)
        super().__init__(*a, **kw)
        self.max_mb = max_microbatch
        self.g_global = torch.zeros_like(self.w_global)

    def round(self):
        _sync(self.dev)
        t0 = time.perf_counter()
        chosen = self._sample()
        if len(chosen) == 0:
            self.round_idx += 1
            return self.ctx.max_scalar(time.perf_counter() - t0), 0
        mine, counts = self._assign(chosen)
        G = len(mine)
        total = float(sum(self.counts[int(c)] for c in chosen))
        self._download(G)
        st, net = self.net.store, self.net
        samples = 0
        if G:
            st.grad[:G].zero_()
            sizes = [self.counts[c] for c in mine]
            same = len(set(sizes)) == 1
            groups = [(0, G)] if same else [(g, g + 1) for g in range(G)]
            for g0, g1 in groups:
                n = sizes[g0]
                idx_all = np.stack([self.client_indices[mine[g]] for g in range(g0, g1)]).astype(np.int32)
                idx_dev = torch.from_numpy(idx_all).to(self.dev)
                lt = self.attack.label_transform_for(mine, net.num_classes) if self.attack else None
                with st.select(g0, g1):
                    for s in range(0, n, self.max_mb):
                        e = min(n, s + self.max_mb)
                        x, y = self.data.batch(idx_dev[:, s:e].contiguous())
                        if lt is not None:
                            y = lt(y, g0, g1)
                        net.train_step(x, y, scale=1.0 / n)
                        samples += (g1 - g0) * (e - s)
        if self.attack is not None and G:
            # model-poisoning attacks act on the reported gradient ("update" = -grad direction)
            self.attack.poison_updates(st.grad[:G], torch.zeros_like(self.w_global), mine)
        coeffs = torch.tensor([self.counts[c] / total for c in mine], dtype=torch.float32,
                              device=self.dev)
        if not getattr(self.aggregator, "needs_all", False):
            self.aggregator(self.ctx, st.grad[:G], coeffs, self.g_global)
        else:
            self.g_global.copy_(self.aggregator(self.ctx, st.grad[:G], counts, self.w_global.numel(),
                                                keys=self._row_keys(counts)))
        # server SGD step (no momentum, as the reference's SGD(lr))
        self.w_global.add_(self.g_global, alpha=-self.lr)
        if G:  # BN running stats from this round's forward passes
            self._mean_buffers(G, coeffs)
        _sync(self.dev)
        dt = self.ctx.max_scalar(time.perf_counter() - t0)
        self.round_idx += 1
        return dt, int(self.ctx.sum_scalar(samples))


class FedSgdWeight(FedAvg):
    """FedSGD exchanging *weights*: one full-batch SGD step per client, then FedAvg. Equals FedSGD
    exactly (sum_k p_k (w - lr g_k) = w - lr sum_k p_k g_k). The reference's homework version
    (homework-1.ipynb:178-230) exchanged gradients under this name."""
    algorithm = "FedSGDWeight"

    def __init__(self, *a, **kw):
        kw["batch_size"] = -1
        kw["local_epochs"] = 1
        super().__init__(*a, **kw)
