"""Simulated Byzantine clients [north-star: the course's announced Part 3 "Attacks & Defenses",
reference README.md:89-92 / lab/README.md:13-16, has no code].

* ``LabelFlip``     — data poisoning: y -> (C - 1 - y) on the malicious clients' batches.
* ``SignFlip``      — model poisoning: the malicious update is negated and scaled,
                      w_k <- w_g - s * (w_k - w_g).
* ``GaussianNoise`` — the malicious update is replaced by N(0, sigma^2) noise.
* ``FreeRider``     — sends back the server weights unchanged (no local work).
"""
from __future__ import annotations

import torch


class Attack:
    def __init__(self, malicious: list[int] | set[int]):
        self.malicious = set(int(m) for m in malicious)

    def label_transform_for(self, slot_clients: list[int], num_classes: int):
        return None

    def poison_updates(self, rows: torch.Tensor, w_global: torch.Tensor, slot_clients: list[int]):
        pass

    def skip_training(self, client: int) -> bool:
        return False

    # RNG state of stochastic attacks, so a resumed run poisons exactly like an uninterrupted one
    def state_dict(self) -> dict:
        return {}

    def load_state_dict(self, sd: dict) -> None:
        pass


class LabelFlip(Attack):
    """Malicious clients train on labels y -> (num_classes - 1 - y). The per-slot flip mask lives
    in ONE persistent device buffer per (device, slot count): each round's transform refreshes it
    (``refresh``, also on its first eager call), so a captured round graph, which reads the buffer,
    replays correctly whichever slots the round's sampling put the attackers in."""

    def __init__(self, malicious):
        super().__init__(malicious)
        self._masks: dict = {}
        self._pinned: list = []  # sources of in-flight mask copies (bounded: trimmed below)

    def _trim(self):
        if len(self._pinned) > 64:
            del self._pinned[:32]  # copies enqueued 32+ rounds ago have long completed

    def label_transform_for(self, slot_clients, num_classes):
        bad = [i for i, c in enumerate(slot_clients) if c in self.malicious]
        if not bad:
            return None
        self._trim()
        n = len(slot_clients)
        mask_cpu = torch.zeros(n, dtype=torch.bool)
        mask_cpu[bad] = True
        fresh: set = set()

        def refresh(device):
            key = (torch.device(device), n)
            if key not in self._masks:
                self._masks[key] = torch.zeros(n, dtype=torch.bool, device=device)
            if key not in fresh:
                src = mask_cpu
                if self._masks[key].is_cuda:
                    # pinned + non-blocking: a pageable copy would make the host wait for the GPU
                    # to drain, serialising rounds that otherwise run unsynchronised (the source
                    # is never written again, so the in-flight copy is safe)
                    src = mask_cpu.pin_memory()
                    self._pinned.append(src)
                self._masks[key].copy_(src, non_blocking=True)
                fresh.add(key)
            return self._masks[key]

        def f(y, g0, g1):
            m = refresh(y.device)[g0:g1]
            return torch.where(m.reshape(-1, *([1] * (y.dim() - 1))), (num_classes - 1) - y, y)
        f.refresh = refresh
        # pure device ops on the persistent mask: a captured round replays it for any slot set
        f.graph_key = ("label_flip", n, num_classes)
        return f


class SignFlip(Attack):
    def __init__(self, malicious, scale: float = 1.0):
        super().__init__(malicious)
        self.scale = scale

    def poison_updates(self, rows, w_global, slot_clients):
        for i, c in enumerate(slot_clients):
            if c in self.malicious:
                rows[i].sub_(w_global).mul_(-self.scale).add_(w_global)


class GaussianNoise(Attack):
    def __init__(self, malicious, sigma: float = 1.0, seed: int = 0):
        super().__init__(malicious)
        self.sigma = sigma
        self.gen = None
        self.seed = seed

    def poison_updates(self, rows, w_global, slot_clients):
        for i, c in enumerate(slot_clients):
            if c in self.malicious:
                if self.gen is None:
                    self.gen = torch.Generator(device=rows.device).manual_seed(self.seed)
                noise = torch.randn(rows.shape[1], generator=self.gen, device=rows.device)
                rows[i].copy_(w_global + self.sigma * noise)

    def state_dict(self):
        return {"gen": None if self.gen is None else self.gen.get_state(),
                "device": None if self.gen is None else str(self.gen.device)}

    def load_state_dict(self, sd):
        if sd.get("gen") is None:
            self.gen = None
            return
        self.gen = torch.Generator(device=sd["device"])
        self.gen.set_state(sd["gen"])


class FreeRider(Attack):
    def skip_training(self, client):
        return client in self.malicious

    def poison_updates(self, rows, w_global, slot_clients):
        for i, c in enumerate(slot_clients):
            if c in self.malicious:
                rows[i].copy_(w_global)


def make_attack(name: str | None, malicious, **kw):
    if not name or name == "none":
        return None
    return {"label_flip": LabelFlip, "sign_flip": SignFlip, "gaussian": GaussianNoise,
            "free_rider": FreeRider}[name](malicious, **kw)
