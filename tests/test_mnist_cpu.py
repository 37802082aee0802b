"""BASELINE configs[0]: the MNIST 2-layer MLP in PyTorch fp32 on the CPU
(CUDA/MNIST_on_GPU/v1.py:35-47), B = 1024, hidden 256 (the reference's) and
128 (configs[1]'s 784x128x10).  Checked against the oracle's fp32 MLP layer,
which is itself bit-exact with the reference's own CPU code v3.c
(tests/test_oracle.py).  torch's CPU GEMM sums in a blocked order, v3.c
strictly in order, so the bar is fp32 rounding: |torch - v3| <= 4e-6 *
sum|x w| + 1e-6 per output (measured max ratio ~1e-7), and the same
argmax wherever the top-2 gap exceeds that bound."""
import numpy as np
import pytest
import torch

from oracle import oracle as O


def _layer_ref(X, W, b, relu):
    B, I = X.shape
    Oo = W.shape[1]
    Y = np.empty((B, Oo), np.float32)
    O.lib().ora_mlp_layer_f32(np.ascontiguousarray(X), np.ascontiguousarray(W), np.ascontiguousarray(b), B, I, Oo,
                              int(relu), Y)
    return Y


@pytest.mark.parametrize("hidden", [256, 128])
def test_mnist_mlp_torch_cpu_matches_v3(hidden):
    from dlq_amd.models import MNISTMLP, mlp_weights, mnist_inputs
    W1, b1, W2, b2 = mlp_weights(hidden=hidden)
    x = mnist_inputs(1024)
    m = MNISTMLP(W1, b1, W2, b2).eval()
    with torch.inference_mode():
        h_t = torch.relu(m.fc1(torch.from_numpy(x))).numpy()
        y_t = m(torch.from_numpy(x)).numpy()
    h = _layer_ref(x, W1, b1, True)
    y = _layer_ref(h, W2, b2, False)
    bound_h = 4e-6 * (np.abs(x) @ np.abs(W1)) + 1e-6
    assert np.all(np.abs(h_t - h) <= bound_h)
    bound_y = 4e-6 * (np.abs(h) @ np.abs(W2)) + 1e-6 + np.abs(W2).sum(0) * bound_h.max(1, keepdims=True)
    assert np.all(np.abs(y_t - y) <= bound_y)
    s = np.sort(y, axis=1)
    clear = (s[:, -1] - s[:, -2]) > 2 * bound_y.max(1)
    assert clear.mean() > 0.9
    assert np.array_equal(y_t.argmax(1)[clear], y.argmax(1)[clear])
