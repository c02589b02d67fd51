"""Reference-named HFL API (lab/tutorial_1a/hfl_complete.py) on the native engine."""
import torch

from ddl25spring_amd.compat import hfl_complete as H
from ddl25spring_amd.models.torch_ref import TorchMnistCnn


def setup_module():
    H.configure(n_train=600, n_test=200)


def test_init_parity_with_reference_constructor():
    torch.manual_seed(10)
    net = H.MnistCnn()
    torch.manual_seed(10)
    tm = TorchMnistCnn()
    from ddl25spring_amd.models import convert
    from ddl25spring_amd.models.zoo import mnist_cnn_mapping
    exported = convert.export_torch(net, tm, mnist_cnn_mapping())
    for k, v in tm.state_dict().items():
        assert torch.equal(exported[k], v), k


def test_split_and_servers_run():
    subsets = H.split(10, True, 10)
    assert len(subsets) == 10 and sum(len(s) for s in subsets) == 600
    res = H.FedAvgServer(0.05, 20, subsets, 0.2, 1, 10).run(2)
    assert res.algorithm == "FedAvg" and res.message_count == [4, 8]
    df = res.as_df()
    assert df["η"].iloc[0] == 0.05 and list(df["Round"]) == [1, 2]
    sgd = H.FedSgdGradientServer(0.05, subsets, 0.2, 10).run(1)
    assert sgd.as_df()["B"].iloc[0] == "∞"
    w = H.FedSgdWeightServer(0.05, subsets, 0.2, 10).run(1)
    assert len(w.test_accuracy) == 1
    non_iid = H.split(5, False, 3)
    assert sorted(sum((list(s.indices) for s in non_iid), [])) == list(range(600))


def test_centralized_and_clients():
    c = H.CentralizedServer(0.05, 100, 1).run(1)
    assert c.message_count == [0]
    subsets = H.split(4, True, 1)
    torch.manual_seed(0)
    server = H.MnistCnn()
    weights = [server.store.data[0].cpu().clone()]
    g = H.GradientClient(subsets[0]).update(weights, 1)
    assert g[0].abs().sum() > 0
    w = H.WeightClient(subsets[0], 0.05, 50, 1).update(weights, 1)
    assert (w[0] - weights[0]).abs().max() > 0
