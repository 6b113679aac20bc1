"""The served armour_main client's protocol, on the CPU with a stand-in server (no GPU needed).

A plain `armour_main <dir>` first asks <dir>/armour.sock (armour_main.cpp, served mode). The request
names the buffer directory as an absolute path, the horizon T and every plan-changing ARMOUR_*
setting of the client, so a server of another horizon or configuration refuses (status 254) and the
client plans in-process. A server that never answers ends the client within
ARMOUR_SERVE_TIMEOUT_MS with -1 in armour.out and a non-zero status; armour.out never keeps a
previous replan's k_opt (KSI/uarmtd_planner.m:202-204 reads it whenever the exit status is 0)."""
import os
import socket
import subprocess
import threading
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "armour-dev_amd", "armour_amd", "armour_main")


def _server(path, reply, requests):
    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    s.bind(path)
    s.listen(4)

    def run():
        c, _ = s.accept()
        buf = b""
        while b"\n" not in buf:
            chunk = c.recv(4096)
            if not chunk:
                break
            buf += chunk
        requests.append(buf.decode())
        if reply is not None:
            c.sendall(bytes([reply]))
            c.close()
        else:
            time.sleep(5)  # never answers within the client's timeout
            c.close()
        s.close()

    th = threading.Thread(target=run, daemon=True)
    th.start()
    return th


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if not k.startswith("ARMOUR_")}
    env.update(kw)
    return env


@pytest.fixture
def bufdir(tmp_path):
    if not os.path.exists(EXE):
        subprocess.run(["make", "-C", os.path.join(ROOT, "armour-dev_amd", "csrc")], check=True, capture_output=True)
    (tmp_path / "armour.in").write_text("0 " * 28 + "0\n")
    (tmp_path / "armour.out").write_text("0.1\n0.2\n0.3\n0.4\n0.5\n0.6\n0.7\n5")  # a previous replan's plan
    return tmp_path


def test_request_names_absolute_dir_horizon_and_settings(bufdir):
    reqs = []
    th = _server(str(bufdir / "armour.sock"), 0, reqs)
    rel = os.path.relpath(str(bufdir), "/tmp")
    r = subprocess.run([EXE, rel], cwd="/tmp", capture_output=True, text=True, timeout=60,
                       env=_env(ARMOUR_NUM_TIME_STEPS="100", ARMOUR_MU_STRATEGY="monotone"))
    th.join(10)
    assert r.returncode == 0, r.stderr  # the stand-in server's status
    d, T, settings = reqs[0].rstrip("\n").split("\t")
    assert d == os.path.realpath(str(bufdir)) and T == "100"
    assert settings == "ARMOUR_MU_STRATEGY=monotone;ARMOUR_NUM_TIME_STEPS=100"
    # the client truncated armour.out before asking: no stale k_opt survives a server that wrote nothing
    assert (bufdir / "armour.out").read_text() == ""


def test_refused_request_plans_in_process(bufdir):
    """status 254 (another T or settings): the client plans itself; without a GPU here that is the
    reference's failure (-1 and a non-zero status), not the server's answer"""
    reqs = []
    th = _server(str(bufdir / "armour.sock"), 254, reqs)
    r = subprocess.run([EXE, str(bufdir)], capture_output=True, text=True, timeout=120, env=_env())
    th.join(10)
    assert len(reqs) == 1
    assert r.returncode != 0
    assert (bufdir / "armour.out").read_text().split() == ["-1"]


def test_silent_server_times_out(bufdir):
    reqs = []
    th = _server(str(bufdir / "armour.sock"), None, reqs)
    t0 = time.time()
    r = subprocess.run([EXE, str(bufdir)], capture_output=True, text=True, timeout=60,
                       env=_env(ARMOUR_SERVE_TIMEOUT_MS="500"))
    dt = time.time() - t0
    th.join(10)
    assert r.returncode != 0 and dt < 4, (r.returncode, dt)
    assert "did not answer" in r.stderr
    assert (bufdir / "armour.out").read_text().split() == ["-1"]
