"""CPU: parameter maps and Adam of the inverse loop (gmm.h:583-706, optimizer.h:13-55)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "3dg-vol-renderer_amd"))
from vr_amd import inverse as inv  # noqa: E402


def test_pack_apply_round_trip_reproduces_covariance():
    rng = np.random.default_rng(0)
    rows = []
    for _ in range(16):
        Q, _ = np.linalg.qr(rng.normal(size=(3, 3)))
        d = rng.uniform(0.01, 0.2, 3) ** 2
        C = Q @ np.diag(d) @ Q.T
        rows.append([*rng.uniform(-1, 1, 3), C[0, 0], C[0, 1], C[0, 2], C[1, 1], C[1, 2], C[2, 2],
                     rng.uniform(0.2, 3), rng.uniform(0.1, 0.9)])
    g = np.array(rows, np.float32)
    p = inv.pack_parameters(g)
    assert p.shape == (16 * 11,)
    back = inv.apply_params(p, [], (0.5, 0.5, 0.5)).gaussians()[:, :11]
    np.testing.assert_allclose(back, g, rtol=2e-5, atol=2e-6)


def test_adam_first_steps_follow_the_reference_formula():
    a = inv.AdamOptimizer(2, lr=0.1)
    x = np.array([1.0, -2.0], np.float32)
    g = np.array([0.5, -4.0], np.float32)
    assert a.step(x, g)
    # t = 1: m = 0.1 g, v = 0.001 g^2, a = lr sqrt(1-0.999)/(1-0.9) -> step = lr * sign(g) (eps aside)
    np.testing.assert_allclose(x, [0.9, -1.9], rtol=1e-5)
    assert not a.step(np.zeros(3, np.float32), np.zeros(3, np.float32))


def test_default_eps_layout():
    e = inv.make_default_eps_for_params(np.zeros(22, np.float32))
    np.testing.assert_array_equal(e[:11], np.float32([0.02] * 3 + [0.1] * 3 + [0.05] * 3 + [0.25, 0.5]))
    np.testing.assert_array_equal(e[11:], e[:11])


def test_sigmoid_pair():
    y = np.float32([0.1, 0.5, 0.9])
    np.testing.assert_allclose(inv.sigmoidf_safe(inv.inv_sigmoidf(y)), y, rtol=1e-6)


def test_sign_vectors_are_balanced_and_keyed():
    a = inv.sign_vector(7, 0, 20000)
    b = inv.sign_vector(7, 1, 20000)
    assert set(np.unique(a)) == {-1.0, 1.0} and abs(a.mean()) < 0.03
    assert not np.array_equal(a, b) and np.array_equal(a, inv.sign_vector(7, 0, 20000))


def test_pack_matches_numpy_eigh_up_to_rotation_sign():
    """The native eigenbasis (Jacobi) gives the LAPACK eigenvalues; apply(pack) is the identity on
    covariances, so any sign choice of the eigenvectors is equivalent."""
    rng = np.random.default_rng(3)
    Q, _ = np.linalg.qr(rng.normal(size=(3, 3)))
    d = np.array([0.01, 0.02, 0.05]) ** 2
    C = Q @ np.diag(d) @ Q.T
    g = np.array([[0, 0, 0, C[0, 0], C[0, 1], C[0, 2], C[1, 1], C[1, 2], C[2, 2], 1.0, 0.5]], np.float32)
    p = inv.pack_parameters(g)
    np.testing.assert_allclose(np.exp(p[6:9]), np.sqrt(np.linalg.eigvalsh(C.astype(np.float32))), rtol=1e-4)
