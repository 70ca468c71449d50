"""shmemx_set_fatal_note: the text registered last is written to stdout and the
process leaves with the registered code when it dies on a fatal signal (the
library's FATAL abort, a GPU fault's abort, a launcher's SIGTERM).  Host-only:
no device call is made."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os, signal, sys
sys.path.insert(0, os.path.join({repo!r}, "openshmem-async_amd"))
import shmem_mi355x as shm
shm.set_fatal_note("first\n", 3)
shm.set_fatal_note({text!r}, {code})
if {uninstall}:
    shm.set_fatal_note(None)
sys.stdout.write("before\n"); sys.stdout.flush()
os.kill(os.getpid(), signal.{sig})
"""


def run_child(sig, text="line {\"value\": 1}\n", code=7, uninstall=False):
    src = CHILD.format(repo=REPO, text=text, code=code, uninstall=uninstall, sig=sig)
    return subprocess.run([sys.executable, "-c", src], capture_output=True, text=True, timeout=120)


@pytest.mark.parametrize("sig", ["SIGABRT", "SIGSEGV", "SIGTERM", "SIGBUS"])
def test_note_written_on_fatal_signal(sig):
    """The note is printed on every fatal signal; a crash of this process
    still exits 128 + signal (a GPU fault during bench extras must not read
    as success), only the launcher's SIGTERM takes the registered code."""
    import signal
    r = run_child(sig)
    want = 7 if sig == "SIGTERM" else 128 + int(getattr(signal, sig))
    assert r.returncode == want, r.stderr
    assert r.stdout == 'before\nline {"value": 1}\n'


def test_empty_note_only_sets_exit_code():
    r = run_child("SIGTERM", text="", code=0)
    assert r.returncode == 0, r.stderr
    assert r.stdout == "before\n"


def test_uninstall_restores_default_disposition():
    r = run_child("SIGTERM", uninstall=True)
    assert r.returncode == -15
    assert r.stdout == "before\n"
