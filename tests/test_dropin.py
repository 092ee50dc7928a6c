"""The drop-in: with dropin/ first on sys.path the reference's own import lines
(pipeline/agent_trainer.py:8-12, Env/drl_engine.py:6-7) resolve to this
package, and the reference's blind-test loop (agent_trainer.py:140-153),
restated verbatim in shape, reproduces the real-data golden trace G1."""
import subprocess
import sys
import textwrap

from conftest import ROOT

SCRIPT = textwrap.dedent(r"""
    import sys
    sys.path.insert(0, {dropin!r})
    import numpy as np, torch
    from models.model import TradingPolicy
    from Env.market_env import FTPEnv
    from Env.drl_engine import DRLEngine, evaluate_individual
    import sgmm_amd
    assert FTPEnv is sgmm_amd.FTPEnv and DRLEngine is sgmm_amd.DRLEngine
    assert TradingPolicy is sgmm_amd.TradingPolicy
    assert evaluate_individual is sgmm_amd.evaluate_individual
    from models.GateUnits import SGU1, SGU2
    from utils.scaler import StandardScaler3D
    import sgmm_amd.gate_units as gu
    assert SGU2 is gu.SGU2 and StandardScaler3D is gu.StandardScaler3D

    d = dict(np.load({golden!r}, allow_pickle=False))
    st = dict(zip(("s1_m", "s1_s", "s2_m", "s2_s"), d["stats"]))
    agent = TradingPolicy()
    agent.set_weights(torch.from_numpy(d["genome"]))
    env = FTPEnv(phi=0.0001, tick_size=0.001, fee_rate=0.0)
    s1, s2, mid, ask, bid, buy_max, sell_min = (d[k] for k in
        ("s1_pred", "s2_pred", "mid", "ask", "bid", "buy_max", "sell_min"))
    inv, cash, rew, fb, fs, acts = [], [], [], [], [], []
    with torch.no_grad():
        for t in range(len(mid)):
            n_s = torch.tensor([[(s1[t] - st["s1_m"]) / st["s1_s"],
                                 (s2[t] - st["s2_m"]) / st["s2_s"],
                                 env.inventory / 2.0]], dtype=torch.float32)
            raw = agent.forward(n_s).squeeze().cpu().numpy()
            a = np.round(raw * 5).astype(int)
            r, info = env.step(a, mid[t], ask[t], bid[t], buy_max[t], sell_min[t], adv_action=None)
            acts.append(a); inv.append(env.inventory); cash.append(env.cash); rew.append(r)
            fb.append(info["fill_buy"]); fs.append(info["fill_sell"])
    acts = np.array(acts)
    assert np.array_equal(acts[:, 0], d["off_a"]) and np.array_equal(acts[:, 1], d["off_b"])
    assert np.array_equal(np.array(inv), d["inventory"])
    assert np.array_equal(np.array(cash), d["cash"]) and np.array_equal(np.array(rew), d["reward"])
    assert np.array_equal(np.array(fb), d["fill_buy"]) and np.array_equal(np.array(fs), d["fill_sell"])
    print("ok", int(np.sum(np.array(fb) | np.array(fs))))
""")


def test_dropin_resolves_reference_imports_and_replays_g1():
    code = SCRIPT.format(dropin=str(ROOT / "dropin"), golden=str(ROOT / "tests/golden/g1_arl_real.npz"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       cwd=str(ROOT / "tests"))
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.strip().startswith("ok")
