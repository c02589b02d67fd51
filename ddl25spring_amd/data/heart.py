"""UCI heart-disease table (1,025 rows x 13 features + binary target) and its preprocessing
recipes / vertical feature partitioners.

The CSV is read from ``DDL_HEART_CSV``, the reference checkout (lab/tutorial_2a/heart.csv) if
mounted, or ``<repo>/data/heart.csv``; nothing is copied. Without any of them a synthetic table
with the same schema, cardinalities and a learnable logistic target is generated (tests say which
one they ran on).

Recipes (reference line numbers):
  * ``centralized_split``  — one-hot(8 categoricals) -> 30 features, train_test_split(0.2),
    MinMax fitted on train (lab/tutorial_2a/centralized.py:33-44)
  * ``vfl_frame``          — MinMax on the 5 numericals of the whole table, one-hot, one-hot
    float target (lab/tutorial_2b/vfl.py:109-115)
  * ``standard_frame``     — one-hot + StandardScaler over features AND target (31 columns,
    generative-modeling.py:137-148, exercise_3.py:150-160)
Partitioners: ``partition_raw_columns`` (D4: raw columns split [3,3,3,4] then expanded to their
one-hot columns -> widths [7,4,6,13]), ``partition_random`` (D5, seeds 42+i), ``partition_balanced``
(D6), ``row_split`` (D7: contiguous 80/20 with .loc semantics).
"""
from __future__ import annotations

import os
from pathlib import Path

import numpy as np
import pandas as pd

CATEGORICAL = ["sex", "cp", "fbs", "restecg", "exang", "slope", "ca", "thal"]
NUMERICAL = ["age", "trestbps", "chol", "thalach", "oldpeak"]
COLUMNS = ["age", "sex", "cp", "trestbps", "chol", "fbs", "restecg", "thalach", "exang", "oldpeak",
           "slope", "ca", "thal", "target"]
_CARD = {"sex": 2, "cp": 4, "fbs": 2, "restecg": 3, "exang": 2, "slope": 3, "ca": 5, "thal": 4}


def _candidates():
    env = os.environ.get("DDL_HEART_CSV")
    if env:
        yield Path(env)
    yield Path("/root/reference/lab/tutorial_2a/heart.csv")
    yield Path(__file__).resolve().parent.parent.parent / "data" / "heart.csv"


def synthetic_heart(n: int = 1025, seed: int = 0) -> pd.DataFrame:
    rng = np.random.default_rng(seed)
    df = pd.DataFrame({
        "age": rng.integers(29, 78, n), "trestbps": rng.integers(94, 200, n),
        "chol": rng.integers(126, 564, n), "thalach": rng.integers(71, 202, n),
        "oldpeak": np.round(rng.uniform(0, 6.2, n), 1)})
    for c, k in _CARD.items():
        df[c] = rng.integers(0, k, n)
    z = (-0.04 * (df.age - 54) + 0.9 * (df.cp > 0) - 0.7 * df.exang - 0.6 * df.oldpeak
         + 0.02 * (df.thalach - 150) - 0.5 * df.ca + 0.8 * (df.thal == 2) - 0.6 * (df.sex == 1) + 0.9)
    df["target"] = (rng.random(n) < 1 / (1 + np.exp(-z))).astype(int)
    return df[COLUMNS]


def load_heart() -> tuple[pd.DataFrame, bool]:
    """-> (frame, is_real)."""
    for p in _candidates():
        if p.is_file():
            return pd.read_csv(p), True
    return synthetic_heart(), False


def centralized_split(df: pd.DataFrame, scaler: str = "minmax", seed: int | None = None):
    from sklearn.model_selection import train_test_split
    from sklearn.preprocessing import MinMaxScaler, StandardScaler
    enc = pd.get_dummies(df, columns=CATEGORICAL)
    X, y = enc.drop("target", axis=1), enc["target"]
    Xtr, Xte, ytr, yte = train_test_split(X, y, test_size=0.2, random_state=seed)
    sc = MinMaxScaler() if scaler == "minmax" else StandardScaler()
    Xtr = sc.fit_transform(Xtr.astype(float))
    Xte = sc.transform(Xte.astype(float))
    return Xtr.astype(np.float32), Xte.astype(np.float32), ytr.values, yte.values


def vfl_frame(df: pd.DataFrame):
    from sklearn.preprocessing import MinMaxScaler
    df = df.copy()
    df[NUMERICAL] = MinMaxScaler().fit_transform(df[NUMERICAL].astype(float))
    enc = pd.get_dummies(df, columns=CATEGORICAL)
    X = enc.drop("target", axis=1)
    Y = pd.get_dummies(enc[["target"]], columns=["target"])
    return X, Y


def standard_frame(df: pd.DataFrame):
    from sklearn.preprocessing import StandardScaler
    enc = pd.get_dummies(df, columns=CATEGORICAL)
    data = pd.concat([enc.drop("target", axis=1), enc["target"]], axis=1)
    scaled = StandardScaler().fit_transform(data.astype(float))
    return pd.DataFrame(scaled, columns=data.columns)


def partition_raw_columns(raw_columns: list[str], encoded_columns: list[str], n_clients: int):
    """D4: split the raw feature columns evenly (last client takes the remainder), then expand
    each categorical to its one-hot columns (substring match on '<name>_', as the reference)."""
    feats = [c for c in raw_columns if c != "target"]
    per = [len(feats) // n_clients] * (n_clients - 1)
    per.append(len(feats) - sum(per))
    out, s = [], 0
    for k in per:
        names = []
        for col in feats[s:s + k]:
            if col not in CATEGORICAL:
                names.append(col)
            else:
                names += [e for e in encoded_columns if "_" in e and col in e]
        out.append(names)
        s += k
    return out


def partition_random(columns: list[str], n_clients: int, seed: int):
    """D5: permutation of the encoded columns with numpy's global seed, split floor/remainder."""
    np.random.seed(seed)
    perm = list(np.random.permutation(columns))
    per = [len(columns) // n_clients] * (n_clients - 1)
    per.append(len(columns) - sum(per))
    out, s = [], 0
    for k in per:
        out.append(perm[s:s + k])
        s += k
    return out


def partition_balanced(columns: list[str], n_clients: int):
    """D6: base = F // n, the first F % n clients get one more column."""
    base, extra = divmod(len(columns), n_clients)
    out, s = [], 0
    for i in range(n_clients):
        k = base + (1 if i < extra else 0)
        out.append(list(columns[s:s + k]))
        s += k
    return out


def row_split(frame: pd.DataFrame, frac: float = 0.8):
    """D7: X.loc[:int(frac*n)] / X.loc[int(frac*n)+1:] (inclusive .loc -> 821 / 204 rows)."""
    cut = int(frac * len(frame))
    return frame.loc[:cut], frame.loc[cut + 1:]
