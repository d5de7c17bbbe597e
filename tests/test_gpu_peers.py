"""GPU parity for per-peer send lists (PeerMap::broadcast_to,
worldql_server/src/transport/peer_map.rs:151-163): the transpose of a tick's CSR with the
disconnected peers dropped, checked against a numpy restatement of the same definition."""
import numpy as np
import pytest

from worldql_server_amd import synth

pytestmark = pytest.mark.gpu


def _expected(offs, peers, n_peers, connected):
    msg = np.repeat(np.arange(len(offs) - 1, dtype=np.uint32), np.diff(offs))
    on = peers < n_peers
    if connected is not None:
        on &= np.unpackbits(connected.view(np.uint8), bitorder="little")[np.minimum(peers, n_peers - 1)] == 1
    p, m = peers[on], msg[on]
    order = np.lexsort((m, p))  # by peer, then message
    p, m = p[order], m[order]
    po = np.searchsorted(p, np.arange(n_peers + 1), side="left").astype(np.uint32)
    return po, m


@pytest.mark.parametrize("frac_connected", [1.0, 0.7, 0.0])
def test_peer_major_matches_transpose(frac_connected):
    import torch
    from worldql_server_amd.router import Router
    w = synth.config_c2(repl_mode="mixed", scale=0.05)
    r = Router(16, 0)
    r.apply_ops(w.ops)
    offs, peers, _ = r.route(w.pos, w.world, w.sender, w.repl)
    M, P = len(offs) - 1, len(peers)
    n_peers = w.n_peers - 7  # a few recipients fall outside: dropped like disconnected peers
    rng = np.random.default_rng(4)
    connected = None
    if frac_connected < 1.0:
        bits = rng.random(((n_peers + 31) // 32) * 32) < frac_connected
        connected = np.packbits(bits, bitorder="little").view(np.uint32)
    dev = torch.device("cuda:0")
    r.set_stream(torch.cuda.current_stream().cuda_stream)
    t_off = torch.from_numpy(offs.view(np.int32)).to(dev)
    t_peers = torch.from_numpy(peers.view(np.int32)).to(dev)
    t_conn = torch.from_numpy(connected.view(np.int32)).to(dev) if connected is not None else None
    po = torch.empty(n_peers + 1, dtype=torch.int32, device=dev)
    mo = torch.empty(max(P, 1), dtype=torch.int32, device=dev)
    r.peer_major_device(t_off.data_ptr(), t_peers.data_ptr(), M, P, t_conn.data_ptr() if t_conn is not None else None,
                        n_peers, po.data_ptr(), mo.data_ptr())
    torch.cuda.synchronize()
    want_po, want_m = _expected(offs, peers, n_peers, connected)
    got_po = po.cpu().numpy().view(np.uint32)
    assert (got_po == want_po).all()
    assert (mo.cpu().numpy().view(np.uint32)[:got_po[-1]] == want_m).all()
    if frac_connected == 0.0:
        assert got_po[-1] == 0
    else:
        assert got_po[-1] > 0
    r.set_stream(None)
