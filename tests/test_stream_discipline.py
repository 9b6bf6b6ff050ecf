"""Static guard for the race class of VERDICT r4 "What's weak" #6 (r04f): a null-stream fill or copy racing the
contexts' non-blocking streams.

Every context stream is created with hipStreamNonBlocking, which does NOT order itself after the null (legacy)
stream.  So inside the library:

- a synchronous hipMemset (null stream) may run before or after work already queued on a context stream:
  forbidden outside the whitelisted self-test entry points;
- hipMemsetAsync / hipMemcpyAsync must name a stream, and never 0 / nullptr / NULL / a default-stream handle;
- a synchronous hipMemcpy is allowed only where nothing queued on a context stream can touch its buffers: after
  a synchronisation earlier in the same function (hipStreamSynchronize / hipEventSynchronize /
  hipDeviceSynchronize / kdpt_synchronize), in an upload of a freshly allocated buffer (dupload), in the
  self tests, or in a helper whose every caller synchronises before calling it (checked one level up).

The check runs on the sources (comments and strings stripped), so a future edit that reintroduces the pattern
fails the CPU suite.
"""
import os
import re

import pytest

from conftest import ROOT

SOURCES = [os.path.join(ROOT, "kdtreepathtraceroptimization_amd", "csrc", f) for f in ("kdpt_runtime.hip", "kd_build.hip")]
SYNC = re.compile(r"\b(hipStreamSynchronize|hipEventSynchronize|hipDeviceSynchronize|kdpt_synchronize)\s*\(")
DEFAULT_STREAMS = {"0", "nullptr", "NULL", "hipStreamLegacy", "hipStreamPerThread", "0u"}
# functions where a synchronous copy or fill is fine by construction
WHITELIST = {
    "dupload": "copies host data into a buffer dalloc has just allocated: nothing can be using it",
}
# helpers whose synchronous copies are fine because every caller synchronises first (checked below)
CALLERS_SYNC = {"check_fault"}


def _strip(src: str) -> str:
    src = re.sub(r"/\*.*?\*/", lambda m: "\n" * m.group(0).count("\n"), src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    return re.sub(r'"(?:\\.|[^"\\])*"', '""', src)


def _functions(src: str):
    """(name, body) of every top-level or namespace-level function definition (brace matching)."""
    out = []
    for m in re.finditer(r"\b([A-Za-z_]\w*)\s*\(([^;{}()]|\([^()]*\))*\)\s*(const\s*)?\{", src):
        name = m.group(1)
        if name in ("if", "for", "while", "switch", "catch", "sizeof", "return", "defined"):
            continue
        start = m.end() - 1
        depth, i = 0, start
        while i < len(src):
            if src[i] == "{":
                depth += 1
            elif src[i] == "}":
                depth -= 1
                if depth == 0:
                    break
            i += 1
        out.append((name, src[start:i + 1], m.start()))
    return out


def _calls(body: str, fn: str):
    """(offset, argument list) of every call of fn in body."""
    res = []
    for m in re.finditer(r"\b" + fn + r"\s*\(", body):
        depth, i, args, cur = 1, m.end(), [], ""
        while i < len(body) and depth:
            ch = body[i]
            if ch == "(":
                depth += 1
            elif ch == ")":
                depth -= 1
                if depth == 0:
                    break
            if ch == "," and depth == 1:
                args.append(cur.strip())
                cur = ""
            else:
                cur += ch
            i += 1
        args.append(cur.strip())
        res.append((m.start(), args))
    return res


def _innermost(funcs, pos):
    best = None
    for name, body, start in funcs:
        end = start + len(body) + 200
        if start <= pos and (best is None or start > best[2]):
            best = (name, body, start)
    return best


@pytest.mark.parametrize("path", SOURCES, ids=os.path.basename)
def test_no_null_stream_fills_or_unsynchronised_copies(path):
    src = _strip(open(path).read())
    funcs = _functions(src)
    bad = []
    for name, body, _ in funcs:
        if name.startswith("kdpt_selftest") or name in WHITELIST:
            continue
        for off, args in _calls(body, "hipMemset"):
            bad.append(f"{name}: synchronous hipMemset (null stream) at +{off}")
        for fn, nargs in (("hipMemsetAsync", 4), ("hipMemcpyAsync", 5)):
            for off, args in _calls(body, fn):
                if len(args) < nargs:
                    bad.append(f"{name}: {fn} without a stream at +{off}")
                elif args[nargs - 1] in DEFAULT_STREAMS:
                    bad.append(f"{name}: {fn} on the default stream ({args[nargs - 1]}) at +{off}")
        for off, args in _calls(body, "hipMemcpy"):
            if name in CALLERS_SYNC:
                continue
            if not SYNC.search(body[:off]):
                bad.append(f"{name}: synchronous hipMemcpy with no synchronisation before it at +{off}")
    assert not bad, "\n".join(bad)


def test_helpers_with_synchronous_copies_are_called_after_a_synchronisation():
    src = _strip(open(SOURCES[0]).read())
    funcs = _functions(src)
    bad = []
    for helper in CALLERS_SYNC:
        for name, body, _ in funcs:
            if name == helper:
                continue
            for off, _ in _calls(body, helper):
                if not SYNC.search(body[:off]):
                    bad.append(f"{name} calls {helper} at +{off} with no synchronisation before it")
    assert not bad, "\n".join(bad)


def test_the_guard_sees_the_pattern():
    """The checker itself: a null-stream fill, a default-stream async copy and an unsynchronised copy are all
    reported, and the synchronised form is not."""
    src = _strip("""
    int f(kdpt_ctx* c) { HIP_TRY(hipMemset(c->image, 0, 4)); return 0; }
    int g(kdpt_ctx* c) { HIP_TRY(hipMemsetAsync(c->image, 0, 4, 0)); return 0; }
    int h(kdpt_ctx* c) { HIP_TRY(hipMemcpy(&x, c->counts, 4, hipMemcpyDeviceToHost)); return 0; }
    int k(kdpt_ctx* c) { HIP_TRY(hipStreamSynchronize(c->stream)); HIP_TRY(hipMemcpy(&x, c->counts, 4, hipMemcpyDeviceToHost)); return 0; }
    """)
    funcs = {n: b for n, b, _ in _functions(src)}
    assert _calls(funcs["f"], "hipMemset")
    assert _calls(funcs["g"], "hipMemsetAsync")[0][1][3] == "0"
    assert not SYNC.search(funcs["h"][:_calls(funcs["h"], "hipMemcpy")[0][0]])
    assert SYNC.search(funcs["k"][:_calls(funcs["k"], "hipMemcpy")[0][0]])
