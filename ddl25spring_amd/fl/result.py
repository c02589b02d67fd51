"""RunResult — byte-compatible with reference hfl_complete.py:113-138 (same fields, same
``as_df`` column names: capitalised keys, "∞" for b == -1, "η" for lr, "Wall time" dropped by
default), plus throughput columns that the reference never recorded."""
from __future__ import annotations

from dataclasses import asdict, dataclass, field

ETA = "\N{GREEK SMALL LETTER ETA}"


@dataclass
class RunResult:
    algorithm: str
    n: int  # number of clients
    c: float  # client fraction
    b: int  # local batch size, -1 == infinity (full local dataset)
    e: int  # local epochs
    lr: float
    seed: int
    wall_time: list[float] = field(default_factory=list)
    message_count: list[int] = field(default_factory=list)
    test_accuracy: list[float] = field(default_factory=list)
    # extensions (not in the reference's table; excluded from as_df unless asked)
    round_time: list[float] = field(default_factory=list, repr=False)
    samples: list[int] = field(default_factory=list, repr=False)
    phase_ms: list[dict] = field(default_factory=list, repr=False)  # per-round device phase times

    def as_df(self, skip_wtime: bool = True, with_throughput: bool = False):
        from pandas import DataFrame
        d = asdict(self)
        extra = {"round_time": d.pop("round_time"), "samples": d.pop("samples")}
        d.pop("phase_ms")
        cols = {k.capitalize().replace("_", " "): v for k, v in d.items()}
        if cols["B"] == -1:
            cols["B"] = "\N{INFINITY}"
        df = DataFrame({"Round": range(1, len(self.wall_time) + 1), **cols})
        df = df.rename(columns={"Lr": ETA})
        if skip_wtime:
            df = df.drop(columns=["Wall time"])
        if with_throughput and extra["round_time"]:
            df["Rounds/s"] = [1.0 / t if t > 0 else float("nan") for t in extra["round_time"]]
            df["Samples/s"] = [s / t if t > 0 else float("nan")
                               for s, t in zip(extra["samples"], extra["round_time"])]
        return df
