"""CPU tests of the C ABI library: it loads, exports every symbol the header
declares (pshmem_* strong, shmem_* weak aliases, reduce-op.c:275-364), the
header compiles and links from C, and the host-side planning logic (which
algorithm, which shards) is right.  No GPU calls here."""
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "shmem_reduce_mi355x.h")
LIBDIR = os.path.join(REPO, "openshmem-async_amd")
LIB = os.path.join(LIBDIR, "libshmem_reduce_mi355x.so")


def declared_functions():
    pre = subprocess.run(["gcc", "-E", "-P", "-x", "c", HEADER], check=True,
                         capture_output=True, text=True).stdout
    return sorted(set(re.findall(r"\b(p?shmemx?_[A-Za-z0-9_]+)\s*\(", pre)))


def exported():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], check=True,
                         capture_output=True, text=True).stdout
    syms = {}
    for line in out.splitlines():
        parts = line.split()
        if len(parts) == 3:
            syms[parts[2]] = (parts[0], parts[1])
    return syms


def test_library_loads(shm):
    assert shm.lib() is not None


def test_every_declared_symbol_is_exported():
    decl = declared_functions()
    assert len(decl) >= 88 + 8
    syms = exported()
    missing = [d for d in decl if d not in syms]
    assert not missing, missing


def test_pshmem_strong_shmem_weak_same_address(shm):
    syms = exported()
    pairs = [f"{t}_{o}_to_all" for t, o in shm.REFERENCE_PAIRS] + ["init", "finalize", "my_pe", "n_pes"]
    assert len(shm.REFERENCE_PAIRS) == 44
    for p in pairs:
        addr_s, kind_s = syms["shmem_" + p]
        addr_p, kind_p = syms["pshmem_" + p]
        assert kind_p == "T" and kind_s == "W", p
        assert addr_s == addr_p, p


def test_reference_pair_set_matches_reduce_op_c(shm, oracle):
    """The 44 (type, op) pairs are exactly those reduce-op.c:388-431 defines."""
    for t in shm.TYPES:
        for o in shm.OPS:
            assert ((t, o) in shm.REFERENCE_PAIRS) == oracle.op_valid(t, o), (t, o)
            assert bool(shm.lib().shmemx_op_valid(shm.TYPES[t], shm.OPS[o])) == oracle.op_valid(t, o)


def test_enum_numbering_matches_oracle(shm, oracle):
    assert shm.TYPES == oracle.TYPES and shm.OPS == oracle.OPS
    for t in shm.TYPES:
        assert shm.type_size(t) == oracle.lib().oracle_type_size(oracle.TYPES[t])


def test_header_compiles_and_links_from_c(tmp_path):
    """A C99 caller written like the reference's users (ISx, isx.c:617)."""
    src = tmp_path / "caller.c"
    src.write_text(r'''
#include <complex.h>
#include "shmem_reduce_mi355x.h"
static long pSync[SHMEM_REDUCE_SYNC_SIZE];
static long long llWrk[SHMEM_REDUCE_MIN_WRKDATA_SIZE];
int main(void) {
    static long long total, mine = 3;
    double complex z = 1.0, w;
    for (int i = 0; i < SHMEM_REDUCE_SYNC_SIZE; i++) pSync[i] = SHMEM_SYNC_VALUE;
    shmem_init();
    shmem_longlong_sum_to_all(&total, &mine, 1, 0, 0, shmem_n_pes(), llWrk, pSync);
    shmem_complexd_prod_to_all(&w, &z, 1, 0, 0, 1, NULL, pSync);
    pshmem_double_max_to_all(NULL, NULL, 0, 0, 0, 1, NULL, pSync);
    shmem_finalize();
    return (int)(total != 3 * shmem_n_pes());
}
''')
    exe = tmp_path / "caller"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.dirname(HEADER), str(src),
                    "-L", LIBDIR, "-lshmem_reduce_mi355x", f"-Wl,-rpath,{LIBDIR}", "-o", str(exe)],
                   check=True)
    assert exe.exists()


REF_SRC = "/root/reference/src"


@pytest.mark.skipif(not os.path.exists(os.path.join(REF_SRC, "shmem.h")),
                    reason="no /root/reference on this host")
def test_reference_header_and_ours_agree(tmp_path):
    """The drop-in boundary against the reference's OWN public headers
    (src/shmem.h, src/pshmem.h, read where they lie; they build standalone):
      * one translation unit includes the reference's shmem.h and pshmem.h and
        then ours: C allows a function to be redeclared only with a compatible
        type, so any of our prototypes that differs from the reference's (the
        44 reductions at shmem.h:1412-1648, their pshmem names, and the
        runtime/collective entry points both headers declare) is a compile
        error under -Werror;
      * the reduction constants our header gives a program (shmem.h:1400-1410)
        equal the reference header's values;
      * a program compiled against the reference's shmem.h alone (no header
        of ours: a reference user's source as it stands) links against
        libshmem_reduce_mi355x.so with every symbol resolved."""
    both = tmp_path / "both.c"
    both.write_text('#include <shmem.h>\n#include <pshmem.h>\n'
                    '#include "shmem_reduce_mi355x.h"\nint main(void){return 0;}\n')
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", REF_SRC,
                    "-I", os.path.dirname(HEADER), "-c", str(both), "-o", str(tmp_path / "both.o")],
                   check=True)
    names = ["SHMEM_REDUCE_SYNC_SIZE", "SHMEM_REDUCE_MIN_WRKDATA_SIZE", "SHMEM_SYNC_VALUE",
             "_SHMEM_REDUCE_SYNC_SIZE", "_SHMEM_REDUCE_MIN_WRKDATA_SIZE", "_SHMEM_SYNC_VALUE"]
    prog = ("#include <stdio.h>\n#include HDR\nint main(void){\n" +
            "".join(f'#ifdef {n}\n printf("{n} %ld\\n", (long)({n}));\n#endif\n' for n in names) +
            "return 0;}\n")
    src = tmp_path / "consts.c"
    src.write_text(prog)
    vals = {}
    for tag, hdr, inc in (("ref", "<shmem.h>", REF_SRC),
                          ("ours", '"shmem_reduce_mi355x.h"', os.path.dirname(HEADER))):
        exe = tmp_path / f"consts_{tag}"
        subprocess.run(["gcc", "-std=c99", f"-DHDR={hdr}", "-I", inc, str(src), "-o", str(exe)],
                       check=True)
        out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
        vals[tag] = dict(line.split() for line in out.splitlines())
    for n in ("SHMEM_REDUCE_SYNC_SIZE", "SHMEM_REDUCE_MIN_WRKDATA_SIZE", "SHMEM_SYNC_VALUE"):
        assert vals["ours"][n] == vals["ref"][n], n
    user = tmp_path / "user.c"
    user.write_text(r'''
#include <shmem.h>
static long pSync[_SHMEM_REDUCE_SYNC_SIZE];
static double dWrk[_SHMEM_REDUCE_MIN_WRKDATA_SIZE];
static long long llWrk[_SHMEM_REDUCE_MIN_WRKDATA_SIZE];
int main(void) {
    static double t[4], s[4];
    static long long total, mine = 1;
    for (int i = 0; i < _SHMEM_REDUCE_SYNC_SIZE; i++) pSync[i] = _SHMEM_SYNC_VALUE;
    shmem_init();
    shmem_double_sum_to_all(t, s, 4, 0, 0, shmem_n_pes(), dWrk, pSync);
    shmem_longlong_sum_to_all(&total, &mine, 1, 0, 0, shmem_n_pes(), llWrk, pSync);
    shmem_barrier_all();
    shmem_finalize();
    return 0;
}
''')
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", REF_SRC, str(user),
                    "-L", LIBDIR, "-lshmem_reduce_mi355x", f"-Wl,-rpath,{LIBDIR}",
                    "-Wl,--no-undefined", "-o", str(tmp_path / "user")], check=True)


def test_header_compiles_as_cpp(tmp_path):
    src = tmp_path / "caller.cpp"
    src.write_text('#include "shmem_reduce_mi355x.h"\n'
                   'int main(){ std::complex<double> a, b; '
                   'shmem_complexd_sum_to_all(&a, &b, 1, 0, 0, 1, nullptr, nullptr); return 0; }\n')
    subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-I", os.path.dirname(HEADER), str(src)],
                   check=True)


# ------------------------------------------------------------------- plans
def test_plan_algorithm_selection(shm):
    P = shm.plan
    # full set, RCCL-native pairs -> RCCL reduce-scatter + all-gather; up to
    # 4 MiB ($SHMEMX_ALLREDUCE_MAX_KB) one RCCL all-reduce
    assert P("double", "sum", 1 << 25, 0, 0, 8, 3, 8).algo == "rccl"
    assert P("double", "sum", (4 << 20) // 8 + 1, 0, 0, 8, 3, 8).algo == "rccl"
    assert P("double", "sum", (4 << 20) // 8, 0, 0, 8, 3, 8).algo == "allreduce"
    assert P("long", "max", 1000, 0, 0, 4, 0, 4).algo == "allreduce"
    assert P("int", "prod", 1000, 0, 0, 2, 1, 2).algo == "allreduce"
    # bitwise (no RCCL op), short (no RCCL type), complex -> A2A
    for t, o in [("long", "xor"), ("int", "and"), ("short", "sum"), ("complexd", "prod")]:
        assert P(t, o, 1000, 0, 0, 4, 2, 4).algo == "a2a", (t, o)
    # float / double / long double min and max: each PE's own fold order
    # (a<b?a:b under NaN and +-0), so GATHER under auto and for an explicit
    # a2a; DIRECT and SIGNAL plan the whole array on every member
    for t in ("float", "double", "longdouble"):
        for o in ("min", "max"):
            assert P(t, o, 1000, 0, 0, 4, 2, 4).algo == "gather", (t, o)
            assert P(t, o, 1000, 0, 0, 4, 2, 4, "a2a").algo == "gather", (t, o)
            for a in ("direct", "signal"):
                q = P(t, o, 1000, 0, 0, 4, 2, 4, a)
                assert q.algo == a and q.chunk == 1000, (t, o, a)
    assert P("double", "min", 1000, 0, 0, 4, 2, 4, "direct").chunk == 1000
    assert P("double", "sum", 1000, 0, 0, 4, 2, 4, "direct").chunk == 250
    # strided or partial sets: A2A under the built-in rule (PE_start bits, no
    # communicator set-up); the set's members-only RCCL communicator
    # (set_comm.cpp) when asked for by name
    assert P("double", "sum", 1000, 0, 1, 4, 2, 8).algo == "a2a"
    assert P("double", "sum", 1000, 1, 0, 3, 2, 8).algo == "a2a"
    assert P("double", "sum", 1 << 20, 1, 0, 3, 2, 8).algo == "a2a"
    assert P("double", "sum", 1000, 1, 0, 3, 2, 8, "rccl").algo == "rccl"
    assert P("double", "sum", 1000, 1, 0, 3, 2, 8, "allreduce").algo == "allreduce"
    assert P("long", "xor", 1000, 1, 0, 3, 2, 8).algo == "a2a"
    assert P("float", "min", 1000, 0, 1, 4, 2, 8).algo == "gather"
    # explicit choices
    assert P("double", "sum", 1000, 0, 0, 4, 2, 4, "gather").algo == "gather"
    assert P("double", "sum", 1000, 0, 0, 4, 2, 4, "a2a").algo == "a2a"
    with pytest.raises(shm.ShmemError) as e:
        P("long", "xor", 1000, 0, 0, 4, 2, 4, "rccl")
    assert e.value.code == 3


def test_plan_errors(shm):
    P = shm.plan
    cases = [((100, 0, 0, 4, 5, 8), 2),      # PE 5 not in {0..3}
             ((100, 1, 1, 3, 2, 8), 2),      # PE 2 not in {1,3,5}
             ((100, 0, 0, 9, 0, 8), 1),      # set beyond npes
             ((-1, 0, 0, 2, 0, 2), 1),       # nreduce < 0
             ((100, 0, -1, 2, 0, 2), 1),     # negative stride
             ((100, 0, 0, 0, 0, 2), 1)]      # empty set
    for args, code in cases:
        with pytest.raises(shm.ShmemError) as e:
            P("double", "sum", *args)
        assert e.value.code == code, args
    assert P("longdouble", "sum", 10, 0, 0, 1, 0, 1).algo in ("a2a", "rccl")
    assert P("longdouble", "max", 10, 0, 0, 4, 1, 4).algo == "gather"   # own order
    assert P("longdouble", "sum", 10, 0, 0, 4, 1, 4).algo == "a2a"   # no RCCL type
    with pytest.raises(shm.ShmemError) as e:
        P("double", "xor", 10, 0, 0, 1, 0, 1)
    assert e.value.code == 1


@pytest.mark.parametrize("t", ["short", "int", "double", "complexd", "complexf"])
@pytest.mark.parametrize("P_", [2, 3, 5, 8])
@pytest.mark.parametrize("n", [0, 1, 7, 64, 1000, 4103, (1 << 25) + 3])
def test_plan_shards_cover_and_align(shm, t, P_, n):
    """A2A shards tile [0, n) exactly, every shard starts on a 16-byte
    boundary of the array; RCCL main+tail == n with 16-byte shards."""
    sz = shm.type_size(t)
    g = max(1, 16 // sz)
    p = shm.plan(t, "sum", n, 0, 0, P_, 0, P_, "a2a")
    assert p.chunk % g == 0 and p.chunk * P_ >= n
    counts = [max(0, min(p.chunk, n - i * p.chunk)) for i in range(P_)]
    assert sum(counts) == n
    assert p.ws_bytes == p.chunk * P_ * sz
    if t in ("int", "double"):
        r = shm.plan(t, "sum", n, 0, 0, P_, 0, P_, "rccl")
        assert r.main == r.chunk * P_ and r.main + r.tail == n
        assert r.chunk % g == 0 and r.tail < P_ * g
    q = shm.plan(t, "sum", n, 0, 0, P_, 0, P_, "gather")
    assert q.ws_bytes == n * P_ * sz


def test_direct_stats_without_calls(shm):
    """shmemx_direct_stats is host-only bookkeeping: no DIRECT call yet means
    zero calls, zero time in every phase and no fences checked, and it never
    needs a device."""
    st = shm.direct_stats(reset=True)
    assert st["calls"] == 0
    assert set(st) == {"calls", *shm.DIRECT_PHASES, *shm.FENCE_STATS, *shm.DIRECT_COUNTS}
    assert all(v == 0 for v in st.values())


def test_typed_stream_forms_for_all_44(shm):
    """shmemx_<T>_<op>_to_all_on_stream exists for every reference pair and
    the header declares it returning int."""
    syms = exported()
    missing = [f"shmemx_{t}_{o}_to_all_on_stream" for t, o in shm.REFERENCE_PAIRS
               if f"shmemx_{t}_{o}_to_all_on_stream" not in syms]
    assert not missing, missing
    pre = subprocess.run(["gcc", "-E", "-P", "-x", "c", HEADER], check=True,
                         capture_output=True, text=True).stdout
    decls = re.findall(r"(\w+)\s+shmemx_\w+_to_all_on_stream\s*\(", pre)
    assert len(decls) == 44 and set(decls) == {"int"}


def test_fortran_constants_match_the_c_header():
    """include/shmem_reduce_mi355x.fh holds the reference's Fortran values
    (src/shmem.fh:63-82): default INTEGER words, twice the C header's long
    counts on LP64; SHMEM_SYNC_VALUE is the same -1."""
    inc = os.path.join(REPO, "include")
    c = dict(re.findall(r"#define\s+(SHMEM_\w+)\s+\(?(-?\d+)L\)?", open(os.path.join(inc, "shmem_reduce_mi355x.h")).read()))
    f = dict(re.findall(r"parameter\s*\(\s*(SHMEM_\w+)\s*=\s*(-?\d+)\s*\)", open(os.path.join(inc, "shmem_reduce_mi355x.fh")).read()))
    assert set(f) == {"SHMEM_REDUCE_SYNC_SIZE", "SHMEM_REDUCE_MIN_WRKDATA_SIZE", "SHMEM_BCAST_SYNC_SIZE",
                      "SHMEM_BARRIER_SYNC_SIZE", "SHMEM_COLLECT_SYNC_SIZE", "SHMEM_SYNC_VALUE"}
    for name, v in f.items():
        want = int(c[name]) if name == "SHMEM_SYNC_VALUE" else 2 * int(c[name])
        assert int(v) == want, (name, v, c[name])


@pytest.mark.parametrize("peers", [False, True])
def test_fold_n_argument_errors_without_a_device(shm, peers):
    """shmemx_fold_n_on_stream / shmemx_fold_n_peers_on_stream reject bad
    arguments before touching HIP: EINVAL for no inputs, a NULL input or a
    pair the reference lacks; nothing to do for zero elements."""
    import ctypes
    fn = shm.lib().shmemx_fold_n_peers_on_stream if peers else shm.lib().shmemx_fold_n_on_stream
    T, O = shm.TYPES, shm.OPS
    ins = (ctypes.c_void_p * 2)(8, None)
    assert fn(T["double"], O["sum"], 8, ins, 0, 16, None) == 1            # nins < 1
    assert fn(T["double"], O["sum"], 8, ins, 2, 16, None) == 1            # NULL input
    assert fn(T["double"], O["xor"], 8, ins, 1, 16, None) == 1            # not a reference pair
    assert fn(T["double"], O["sum"], 8, ins, 2, 0, None) == 0             # zero elements


def test_fused_twoshot_limit_setter(shm):
    """shmemx_set_fused_twoshot_kb returns the previous limit (the 4 MiB
    default unless $SHMEMX_FUSED_TWOSHOT_KB says otherwise) and refuses a
    negative one."""
    import os
    default = int(os.environ.get("SHMEMX_FUSED_TWOSHOT_KB", "4096"))
    prev = shm.set_fused_twoshot_kb(0)
    assert prev == default
    assert shm.set_fused_twoshot_kb(16384) == 0
    with pytest.raises(shm.ShmemError):
        shm.set_fused_twoshot_kb(-1)
    assert shm.set_fused_twoshot_kb(prev) == 16384


def test_plan_without_set_comms():
    """$SHMEMX_SET_COMMS=0 (read once per process, so in a child): partial
    sets plan A2A for the RCCL-native pairs and refuse an explicit rccl, as
    before set communicators existed; the whole job is unchanged."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); import shmem_mi355x as shm\n"
            "assert shm.plan('double', 'sum', 1000, 1, 0, 3, 2, 8).algo == 'a2a'\n"
            "assert shm.plan('double', 'sum', 1000, 0, 0, 8, 2, 8).algo == 'allreduce'\n"
            "try:\n    shm.plan('double', 'sum', 1000, 1, 0, 3, 2, 8, 'rccl')\n    raise SystemExit('rccl planned')\n"
            "except shm.ShmemError as e:\n    assert e.code == 3\n"
            "print('ok')\n") % os.path.join(os.path.dirname(HEADER), "..", "openshmem-async_amd")
    out = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, SHMEMX_SET_COMMS="0"),
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stdout + out.stderr
