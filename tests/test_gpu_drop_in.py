"""The drop-in executable armour_main speaks the reference's file protocol
(kinova_planner_realtime/armour_main.cu:5-10, 37-77, 319-398)."""
import os
import subprocess

import numpy as np
import pytest

import armour_amd as A
from armour_amd.robots import KINOVA

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "armour-dev_amd", "armour_amd", "armour_main")


def write_input(path, world):
    """the writer of KSI/uarmtd_planner.m:169-196 (%.10f, space separated)"""
    q0, qd0, qdd0, qdes, obs = world
    with open(os.path.join(path, "armour.in"), "w") as f:
        for v in (q0, qd0, qdd0, qdes):
            f.write(" ".join(f"{x:.10f}" for x in v) + "\n")
        f.write(f"{len(obs)}\n")
        for o in obs:
            f.write(" ".join(f"{x:.10f}" for x in o) + "\n")


def run(path, T):
    env = dict(os.environ, ARMOUR_NUM_TIME_STEPS=str(T))
    return subprocess.run([EXE, path], env=env, capture_output=True, text=True, timeout=300)


def test_example_world_protocol(tmp_path):
    T = 20
    world = A.example_world()
    write_input(str(tmp_path), world)
    r = run(str(tmp_path), T)
    assert r.returncode == 0, r.stderr
    out = [float(v) for v in open(tmp_path / "armour.out").read().split()]
    # the same problem through the library (inputs rounded as the text file carries them)
    rounded = [np.round(np.asarray(a, dtype=np.float64), 10) for a in world]
    P = A.Planner(T=T, max_obstacles=10, max_worlds=1)
    res, _ = P.plan([tuple(rounded)])
    if res[0]["feasible"]:
        assert len(out) == 8
        np.testing.assert_allclose(out[:7], res[0]["k_opt"], rtol=1e-9, atol=1e-9)
    else:
        assert out[0] == -1 and len(out) == 2
    NJ = 7
    c = np.loadtxt(tmp_path / "armour_joint_position_center.out")
    assert c.shape == (T * NJ, 3)
    np.testing.assert_allclose(c.reshape(T, NJ, 3), P.link_centers(0), rtol=1e-9, atol=1e-9)
    g = np.loadtxt(tmp_path / "armour_joint_position_radius.out")
    assert g.shape == (T * NJ * 3, 6)
    np.testing.assert_allclose(g.reshape(T, NJ, 3, 6), P.link_generators(0), rtol=1e-9, atol=1e-12)
    u = np.loadtxt(tmp_path / "armour_control_input_radius.out")
    assert u.shape == (T, 7)
    np.testing.assert_allclose(u, P.torque_radius(0), rtol=1e-9)
    cons = np.loadtxt(tmp_path / "armour_constraints.out")
    m = P.num_constraints(10)
    assert cons.shape == (m + 28,)
    np.testing.assert_allclose(cons[:m], P.constraints(0), rtol=1e-5, atol=1e-5)
    b = P.joint_bounds()
    np.testing.assert_allclose(cons[m:], b, rtol=1e-5)
    # the reference's writers are ofstreams at setprecision(10) / (6) (armour_main.cu:319-398): every
    # number is printf's %.10g / %.6g rendering of itself, space / newline separated as there
    for name, prec in (("armour_joint_position_center.out", 10), ("armour_joint_position_radius.out", 10),
                       ("armour_control_input_radius.out", 10), ("armour_constraints.out", 6)):
        text = open(tmp_path / name).read()
        toks = text.split()
        assert toks and all(t == "%.*g" % (prec, float(t)) for t in toks), name
        if prec == 10:
            assert all(line.endswith(" ") for line in text.splitlines()), name
    # per joint [lb + qe, ub - qe], then [-v + qde, v - qde] (armour_main.cu:385-396)
    assert np.all(b[0:14:2] > KINOVA.state_lb) and np.all(b[1:14:2] < KINOVA.state_ub)
    np.testing.assert_allclose(b[14::2], -b[15::2])
    assert np.all(b[15::2] < KINOVA.speed_limits)


def test_missing_input_fails_like_reference(tmp_path):
    r = run(str(tmp_path), 10)
    assert r.returncode != 0
    assert open(tmp_path / "armour.out").read().split() == ["-1"]


def test_too_many_obstacles_fails_like_reference(tmp_path):
    world = A.make_world(0, 3)
    q0, qd0, qdd0, qdes, obs = world
    write_input(str(tmp_path), (q0, qd0, qdd0, qdes, np.tile(obs, (14, 1))))  # 42 > MAX_OBSTACLE_NUM
    r = run(str(tmp_path), 10)
    assert r.returncode != 0
    assert open(tmp_path / "armour.out").read().split() == ["-1"]


def _outputs(path):
    names = ["armour.out", "armour_joint_position_center.out", "armour_joint_position_radius.out",
             "armour_control_input_radius.out", "armour_constraints.out"]
    return {n: open(os.path.join(path, n)).read() for n in names}


def test_served_mode_matches_in_process(tmp_path):
    """`armour_main --serve` keeps one planner warm; a plain armour_main run then forwards its
    buffer directory over <buffer>/armour.sock and exits with the server's status. The five output
    files must be byte-identical to an in-process run, failures included, and a served replan
    skips process-wide HIP initialisation."""
    import time

    T = 20
    srv, loc = tmp_path / "srv", tmp_path / "loc"
    srv.mkdir()
    loc.mkdir()
    env = dict(os.environ, ARMOUR_NUM_TIME_STEPS=str(T))
    server = subprocess.Popen([EXE, "--serve", str(srv)], env=env, stdout=subprocess.DEVNULL,
                              stderr=subprocess.PIPE, text=True)
    try:
        for _ in range(600):
            if (srv / "armour.sock").exists() or server.poll() is not None:
                break
            time.sleep(0.1)
        assert server.poll() is None and (srv / "armour.sock").exists(), "server did not start"
        worlds = [A.example_world(), A.make_world(3, 10, profile="survey"), A.make_world(4, 10, profile="survey")]
        walls = []
        for world in worlds:
            write_input(str(srv), world)
            write_input(str(loc), world)
            t0 = time.perf_counter()
            rs = run(str(srv), T)
            walls.append((time.perf_counter() - t0) * 1e3)
            rl = subprocess.run([EXE, str(loc)], env=dict(env, ARMOUR_NO_SERVE="1"), capture_output=True, text=True,
                                timeout=300)
            assert rs.returncode == 0 and rl.returncode == 0, (rs.stderr, rl.stderr)
            os_, ol = _outputs(str(srv)), _outputs(str(loc))
            # the reported planning time (last line of armour.out) differs run to run
            assert os_["armour.out"].split()[:-1] == ol["armour.out"].split()[:-1]
            for n in list(os_)[1:]:
                assert os_[n] == ol[n], n
        # an error is served like the in-process run: -1 and a non-zero status
        q0, qd0, qdd0, qdes, obs = A.make_world(0, 3)
        write_input(str(srv), (q0, qd0, qdd0, qdes, np.tile(obs, (14, 1))))
        r = run(str(srv), T)
        assert r.returncode != 0 and open(srv / "armour.out").read().split() == ["-1"]
        print(f"served armour_main wall time: {[round(w, 1) for w in walls]} ms")
        assert min(walls) < 100
    finally:
        server.terminate()
        server.wait(timeout=30)
    assert not (srv / "armour.sock").exists()


def test_served_late_plan_is_discarded(tmp_path):
    """A client that times out (ARMOUR_SERVE_TIMEOUT_MS) writes -1 and exits non-zero; the server's
    plan for it finishes later (ARMOUR_SERVE_DELAY_MS holds it back here) and must not land in the
    buffer directory: the server commits its .part files only while the client still waits, under
    the directory's lock. The next replan is served normally."""
    import time

    T = 20
    srv = tmp_path / "srv"
    srv.mkdir()
    env = dict(os.environ, ARMOUR_NUM_TIME_STEPS=str(T))
    server = subprocess.Popen([EXE, "--serve", str(srv)], env=dict(env, ARMOUR_SERVE_DELAY_MS="1500"),
                              stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    try:
        for _ in range(600):
            if (srv / "armour.sock").exists() or server.poll() is not None:
                break
            time.sleep(0.1)
        assert server.poll() is None and (srv / "armour.sock").exists(), "server did not start"
        write_input(str(srv), A.example_world())
        r = subprocess.run([EXE, str(srv)], env=dict(env, ARMOUR_SERVE_TIMEOUT_MS="300"), capture_output=True,
                           text=True, timeout=60)
        assert r.returncode != 0 and "did not answer" in r.stderr
        time.sleep(3.0)  # the server's plan has finished by now, and was discarded
        assert open(srv / "armour.out").read().split() == ["-1"]
        assert not any(p.name.endswith(".part") for p in srv.iterdir())
        assert not (srv / "armour_constraints.out").exists()
        # a client that waits long enough gets the plan
        r = subprocess.run([EXE, str(srv)], env=dict(env, ARMOUR_SERVE_TIMEOUT_MS="20000"), capture_output=True,
                           text=True, timeout=60)
        assert r.returncode == 0, r.stderr
        assert len(open(srv / "armour.out").read().split()) in (2, 8)
        assert (srv / "armour_constraints.out").exists()
    finally:
        server.terminate()
        server.wait(timeout=30)


def test_single_world_entry_matches_batch():
    """armour_plan (SURVEY.md §8(b)'s single-world entry, which armour_main calls) gives the plan and
    the five .out payloads of armour_plan_batch with one world and the getters, bitwise"""
    import numpy as np

    world = A.make_world(11, 20, profile="survey")
    P = A.Planner(T=128, max_obstacles=20, max_worlds=1)
    r1, _, outs = P.plan_one(world)
    (r0,), _ = P.plan([world])
    assert np.array_equal(r0["k_opt"], r1["k_opt"]) and r0["feasible"] == r1["feasible"]
    assert (r0["status"], r0["iterations"], r0["evaluations"]) == (r1["status"], r1["iterations"], r1["evaluations"])
    assert np.array_equal(outs["constraints"], P.constraints(0))
    assert np.array_equal(outs["link_centers"].ravel(), P.link_centers(0).ravel())
    assert np.array_equal(outs["torque_radius"].ravel(), P.torque_radius(0).ravel())
    assert np.array_equal(outs["link_generators"].ravel(), P.link_generators(0).ravel())
