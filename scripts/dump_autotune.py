"""Print the conv autotuner's picks for the headline ResNet-18 step at 1, 2, 4 and 8 clients per GPU
(one warm-up FedAvg round each on a small synthetic set), as 'mode G HxW C->K stride cfg splits'.

    python scripts/dump_autotune.py > gpurun_out/autotune.txt
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def decode(cfg):
    if not cfg:
        return "heuristic"
    bp, bq, bk, ns = (cfg & 0xff) * 16, ((cfg >> 8) & 0xff) * 16, (cfg >> 16) & 0xff, (cfg >> 24) & 0xff
    return f"{bp}x{bq}x{bk}s{ns & 0x3f}{'H' if ns & 0x40 else ''}"


def main():
    from ddl25spring_amd.data.images import DeviceImageDataset, synthetic_images
    from ddl25spring_amd.data.split import split
    from ddl25spring_amd.fl.algorithms import FedAvg
    from ddl25spring_amd.models import resnet18_cifar
    from ddl25spring_amd.ops import autotune
    from ddl25spring_amd.runtime import dist as rdist
    ctx = rdist.init()
    for G in (1, 2, 4, 8):
        train = synthetic_images("cifar10", 1000 * G, seed=0)
        data = DeviceImageDataset(train, ctx.device)
        parts = split(G, True, 10, labels=train.labels)
        fl = FedAvg(resnet18_cifar, data, parts, lr=0.01, batch_size=100, client_fraction=1.0,
                    seed=10, eval_every=0)
        fl.round()
    for key, (cfg, sp) in sorted(autotune.cache().items(), key=lambda kv: (kv[0][1], kv[0][0], -kv[0][3])):
        mode, G, N, H, W, C, K, R, S, st, pad, flags = key
        print(f"{mode:5s} G{G} N{N} {H}x{W} {C}->{K} k{R} s{st} flags{flags} -> {decode(cfg)} splits={sp}")


if __name__ == "__main__":
    main()
