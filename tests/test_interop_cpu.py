"""safetensors checkpoints with tch VarStore naming, host-only.

The file format is checked against the official `safetensors` package (read
and write); the tch naming (root-path names, "__<count>" suffix on repeats,
conv/linear create `bias` before `weight`: interop.cpp kModuleOrder) is
restated from tch 0.13, which is not vendored: parity unpinned."""
import os

import numpy as np
import pytest

spai = pytest.importorskip("spai")
st = pytest.importorskip("safetensors.numpy")


def tch_names(modules):
    """flat-order names for a list of modules ("conv", "bn", "linear"): tch creates
    conv/linear `bias` before `weight` (the suffix counts variables created so
    far); the flat vector stores weight before bias"""
    names, seen = [], set()

    def name(base):
        n = base + "__%d" % created[0] if base in seen else base
        seen.add(base)
        created[0] += 1
        return n

    created = [0]
    for m in modules:
        if m == "bn":
            names += [name(v) for v in ("weight", "bias", "running_mean", "running_var")]
        else:
            b = name("bias")
            w = name("weight")
            names += [w, b]
    return names


def expected_names(blocks):
    """stem + 2*blocks residual convs (conv, BN), policy head (conv, BN, linear), value head"""
    return tch_names(["conv", "bn"] * (1 + 2 * blocks) + ["conv", "bn", "linear", "conv", "bn", "linear"])


@pytest.mark.parametrize("blocks", [0, 2, 6])
def test_safetensors_roundtrip_and_format(tmp_path, blocks):
    p = spai.init_params(blocks, 64, seed=blocks + 1)
    path = str(tmp_path / "ckpt.safetensors")
    spai.save_params(path, p, blocks)
    np.testing.assert_array_equal(spai.load_params(path, blocks), p)
    # the official reader sees tch's names and shapes, in construction order
    t = st.load_file(path)
    names = expected_names(blocks)
    assert set(t) == set(names)
    flat = np.concatenate([t[n].reshape(-1) for n in names])
    np.testing.assert_array_equal(flat, p)
    assert t["weight"].shape == (64, 3, 3, 3) and t["bias"].shape == (64,)   # stem conv (bias created first)
    assert names[:6] == ["weight", "bias", "weight__2", "bias__3", "running_mean", "running_var"]
    assert t["running_var"].shape == (64,)
    last_lin = names[-2]
    assert t[last_lin].shape == (1, 126)                       # value head linear
    assert t[names[-2 - 6 - 2]].shape == (7, 1344)             # policy head linear


def test_safetensors_load_foreign_file(tmp_path):
    """a file written by the safetensors package (any tensor order) loads by name"""
    blocks = 1
    p = spai.init_params(blocks, 64, seed=3)
    ref = os.path.join(tmp_path, "ref.safetensors")
    spai.save_params(ref, p, blocks)
    t = st.load_file(ref)
    other = os.path.join(tmp_path, "other.safetensors")
    st.save_file({k: t[k] for k in sorted(t, reverse=True)}, other, metadata={"format": "pt"})
    np.testing.assert_array_equal(spai.load_params(other, blocks), p)


def test_safetensors_errors(tmp_path):
    blocks = 1
    p = spai.init_params(blocks, 64, seed=3)
    path = str(tmp_path / "a.safetensors")
    spai.save_params(path, p, blocks)
    with pytest.raises(spai.SpaiError):           # wrong architecture (missing tensors)
        spai.load_params(path, 2)
    t = st.load_file(path)
    t["weight"] = t["weight"][:32]                 # wrong shape
    bad = str(tmp_path / "bad.safetensors")
    st.save_file(t, bad)
    with pytest.raises(spai.SpaiError):
        spai.load_params(bad, blocks)
    t = st.load_file(path)
    t["bias"] = t["bias"].astype(np.float64)       # wrong dtype
    st.save_file(t, bad)
    with pytest.raises(spai.SpaiError):
        spai.load_params(bad, blocks)
    with pytest.raises(spai.SpaiError):
        spai.load_params(str(tmp_path / "missing.safetensors"), blocks)



def test_safetensors_ttt_and_chess_nets(tmp_path):
    """the TicTacToe (model/tictactoe.rs) and chess (model/chess.rs) nets: round trip, and the
    official reader sees tch names/shapes whose construction-order concatenation is the flat vector"""
    import spai_chess
    import spai_ttt
    p = spai_ttt.init_params(2, 4)
    path = str(tmp_path / "ttt.safetensors")
    spai.save_params(path, p, 2, game=spai.GAME_TICTACTOE)
    np.testing.assert_array_equal(spai.load_params(path, 2, game=spai.GAME_TICTACTOE, n=p.size), p)
    t = st.load_file(path)
    names = expected_names(2)
    assert set(t) == set(names)
    np.testing.assert_array_equal(np.concatenate([t[n].reshape(-1) for n in names]), p)
    assert t["weight"].shape == (64, 3, 3, 3) and t[names[-2]].shape == (1, 27)
    assert t[names[-2 - 6 - 2]].shape == (9, 288)

    blocks = 1
    p = spai_chess.init_params(blocks, 2)
    path = str(tmp_path / "chess.safetensors")
    spai.save_params(path, p, blocks, hidden=256, game=spai.GAME_CHESS)
    np.testing.assert_array_equal(spai.load_params(path, blocks, hidden=256, game=spai.GAME_CHESS, n=p.size), p)
    t = st.load_file(path)
    names = tch_names(["conv", "bn"] * (1 + 2 * blocks) + ["conv"] * 3 + ["linear"] * 2)
    assert set(t) == set(names)
    np.testing.assert_array_equal(np.concatenate([t[n].reshape(-1) for n in names]), p)
    shapes = [t[n].shape for n in names]
    assert shapes[0] == (256, 19, 3, 3)
    assert shapes[-10:] == [(256, 256, 1, 1), (256,), (73, 256, 1, 1), (73,), (1, 256, 1, 1), (1,),
                            (256, 64), (256,), (1, 256), (1,)]
    with pytest.raises(spai.SpaiError):      # wrong count for the architecture
        spai.save_params(path, p[:-1], blocks, hidden=256, game=spai.GAME_CHESS)
