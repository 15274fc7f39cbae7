"""The code-parity bar shared by the GPU tests (test infrastructure):
bit-exact ids, and on the first divergent code a verdict from
tests/divergence.py -- an fp near-tie (the reference's own draw there sits
within rounding of a decision boundary) or a bug."""
import numpy as np

from divergence import classify, describe

# the oracle replays the utterance up to the divergent frame on the CPU; past
# this frame the verdict is left to tools/classify_divergence.py (offline)
CLASSIFY_MAX_FRAME = 48


def codes_equal(got, want, what, ctx=None):
    """ctx (optional): dict(oracle, ids, spk, lang, params) of the utterance
    -- the oracle's keyword parameters -- to classify a divergence."""
    assert got is not None, what
    assert got.shape == want.shape, (what, got.shape, want.shape)
    bad = np.argwhere(got != want)
    if not len(bad):
        return
    f, g = (int(v) for v in bad[0])
    msg = (f"{what}: first divergent code at frame {f} group {g} "
           f"(got {got[f, g]}, reference {want[f, g]}; {len(bad)} codes differ)")
    if ctx is not None:
        if f > ctx.get("max_frame", CLASSIFY_MAX_FRAME):
            msg += f"; unclassified here (frame {f}: run tools/classify_divergence.py)"
        else:
            try:
                msg += "; " + describe(classify(ctx["oracle"], ctx["ids"], ctx["spk"], ctx["lang"], f, g,
                                                ctx["params"], got=int(got[f, g])))
            except Exception as e:   # the verdict is a diagnostic: never mask the failure itself
                msg += f"; classification failed ({e!r})"
    raise AssertionError(msg)


def codes_equal_upto_classified(got, want, what, known):
    """The bar for very long runs, where some draw of tens of thousands sits
    within rounding of a boundary: the codes are bit-exact up to the first
    divergence, and that divergence is one recorded in the fixture's manifest
    entry (`known`: [{frame, group, got, verdict, record}]) with an
    "fp near-tie" verdict from tools/classify_divergence.py.  Any other
    divergence fails (a kernel change that moves it must be re-classified).
    Returns the first divergent frame (None: no divergence)."""
    assert got is not None, what
    assert got.shape == want.shape, (what, got.shape, want.shape)
    bad = np.argwhere(got != want)
    if not len(bad):
        return None
    f, g = (int(v) for v in bad[0])
    for k in known or []:
        if (k["frame"], k["group"], k["got"]) == (f, g, int(got[f, g])) and k["verdict"].startswith("fp near-tie"):
            return f
    raise AssertionError(f"{what}: first divergent code at frame {f} group {g} (got {got[f, g]}, reference "
                         f"{want[f, g]}; {len(bad)} codes differ) -- not a recorded near-tie: run "
                         f"tools/classify_divergence.py")
