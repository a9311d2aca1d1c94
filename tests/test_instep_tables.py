"""The in-step variant choice (tools/ab/instep_tables.py, CPU): runner-up tables from the tuner's top list, and the
per-key pick over step profiles (only a clear win over the committed choice switches), on synthetic tables."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(REPO, "tools", "ab", "instep_tables.py")
K1 = [0, 1, 72, 96, 320, 72, 96, 320, 3, 1, False, 2880]
K2 = [0, 1, 36, 48, 640, 36, 48, 640, 3, 1, False, 5760]


def _table(path, entries):
    path.write_text(json.dumps([{"key": k, "algo": a, "splitk": s} for k, a, s in entries]))


def _load(path):
    return {tuple(e["key"]): (e["algo"], e["splitk"]) for e in json.loads(path.read_text())}


def test_make_runner_up_tables(tmp_path):
    base, top = tmp_path / "base.json", tmp_path / "top.json"
    _table(base, [(K1, 33, 1), (K2, 31, 3)])
    # the committed choice may appear in the top list: it is skipped
    top.write_text(json.dumps([{"key": K1, "top": [[47, 1, 27.3], [33, 1, 30.2], [62, 1, 31.8]]},
                               {"key": K2, "top": [[47, -2, 30.8], [31, 3, 33.2]]}]))
    subprocess.run([sys.executable, TOOL, "make", str(base), str(top), str(tmp_path / "alt"), "2"], check=True,
                   capture_output=True)
    a1, a2 = _load(tmp_path / "alt1.json"), _load(tmp_path / "alt2.json")
    assert a1[tuple(K1)] == (47, 1) and a1[tuple(K2)] == (47, -2)
    assert a2[tuple(K1)] == (62, 1) and a2[tuple(K2)] == (31, 3)   # K2 has one runner-up: committed kept
    subprocess.run([sys.executable, TOOL, "make", str(base), str(top), str(tmp_path / "skip"), "1", "1"], check=True,
                   capture_output=True)
    assert _load(tmp_path / "skip1.json")[tuple(K1)] == (62, 1)


def test_pick_only_clear_wins(tmp_path):
    base, alt = tmp_path / "base.json", tmp_path / "alt1.json"
    _table(base, [(K1, 33, 1), (K2, 31, 3)])
    _table(alt, [(K1, 47, 1), (K2, 47, -2)])
    kc, ka = tmp_path / "keys_c.json", tmp_path / "keys_a.json"
    # step time per key: [launches, us, (algo, split) it ran]; K1 1 % faster (kept committed), K2 15 % faster
    kc.write_text(json.dumps({json.dumps(K1): [14, 400.0, [33, 1]], json.dumps(K2): [12, 372.5, [31, 3]]}))
    ka.write_text(json.dumps({json.dumps(K1): [14, 396.0, [47, 1]], json.dumps(K2): [12, 316.0, [47, -2]]}))
    out = tmp_path / "out.json"
    r = subprocess.run([sys.executable, TOOL, "pick", str(base), str(out), str(kc), str(alt), str(ka)], check=True,
                       capture_output=True, text=True)
    t = _load(out)
    assert t[tuple(K1)] == (33, 1) and t[tuple(K2)] == (47, -2)
    assert "1 shapes changed" in r.stdout
