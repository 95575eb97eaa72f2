"""bench.py --gpus N: the parent starts torch.distributed.run with N ranks as a child process
and relays rank 0's line.  Exercised with the CPU stand-in step on gloo (no GPU here)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, timeout=240):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_launcher_two_ranks():
    r = _run("--gpus", "2", "--standin", "cpu", "--steps", "3", "--warmup", "1")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout          # only rank 0 prints
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2
    assert rec["config"]["parallelism"] == "shard2"
    assert rec["steps"] == 3


def test_world_mismatch_refused():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--standin", "cpu"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_main_does_not_shadow_module_functions():
    """bench.main() dispatches to module-level functions (bench_c5, bench_compress, ...); a local
    import of the same name inside main() would make those calls fail at run time."""
    import ast
    src = open(os.path.join(ROOT, "bench.py")).read()
    tree = ast.parse(src)
    top = {f.name for f in tree.body if isinstance(f, ast.FunctionDef)}
    main = next(f for f in tree.body if isinstance(f, ast.FunctionDef) and f.name == "main")
    local = set()
    for n in ast.walk(main):
        if isinstance(n, (ast.Import, ast.ImportFrom)):
            local |= {(a.asname or a.name).split(".")[0] for a in n.names}
        elif isinstance(n, ast.Name) and isinstance(n.ctx, ast.Store):
            local.add(n.id)
    assert not (local & top), f"main() shadows module functions: {sorted(local & top)}"


def test_c5_one_corpus_split_into_distinct_rounds_at_every_n():
    """bench's c5 leg (tools/bench_c5.py) is strong scaling over ONE corpus: 400 GiB of blocks
    drawn from one seed, split over the ranks by bytes, each share cut into rounds of at most
    16 GiB; at every N the rounds of all ranks tile the corpus once (no block decoded twice)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import numpy as np
    import bench_c5
    from gobeansdb_amd import shard
    sizes, is_text = bench_c5.corpus(400.0)
    assert sizes.sum() >= 400 * 2**30 and sizes[:-1].sum() < 400 * 2**30
    assert sizes.min() >= 4096 and sizes.max() <= 65536
    assert abs(is_text.mean() - 0.7) < 0.01
    s2, t2 = bench_c5.corpus(400.0)
    assert np.array_equal(sizes, s2) and np.array_equal(is_text, t2)   # the same on every rank
    for world in (1, 2, 4, 8):
        covered = []
        for lo, hi in shard.partition_by_bytes(sizes, world):
            rounds = bench_c5.plan_rounds(sizes, lo, hi, 16.0)
            assert all(int(sizes[a:b].sum()) <= 16 * 2**30 + 65536 for a, b in rounds)
            covered += rounds
        assert covered[0][0] == 0 and covered[-1][1] == len(sizes)
        assert all(x[1] == y[0] for x, y in zip(covered, covered[1:]))
        assert len(covered) <= 25 + world
