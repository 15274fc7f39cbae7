"""Classify a code divergence from the reference as an fp near-tie or a bug
(TEST INFRASTRUCTURE).

The GPU path sums every dot product in a different order from the
reference's scalar loops (K.c:139-148), so its logits differ from the
reference's by rounding: each logit of a GEMV within 2e-6 * sum_k |a_k x_k| +
1e-6 (the bar of tests/test_gpu_kernels.py).  Ids stay bit-exact as long as no
draw sits closer than that to one of its decision boundaries.  When a test
finds a first divergent code at (frame f, group g), this module asks how close
the REFERENCE's own draw there was to flipping:

1. the oracle port (bit-exact to the reference's build, tests/test_oracle_*.py)
   replays the utterance up to frame f with a trace armed on draw (f, g)
   (`Oracle.trace_draw`): the logits handed to the sampler, the logit head's
   input row x, the RNG state before the draw and the drawn id -- the same
   record oracle/ref_driver.c keeps of the reference's sampler calls;
2. `flip_distance` restates the fast top-k draw of K.c:407-484 (the path
   every default / greedy draw takes) and returns the smallest uniform
   perturbation eps of the raw logits (|d_i| <= eps for every i) that changes
   the drawn id: the cumulative-sum boundaries either side of r = u * sum
   (for weights w_j = exp((l_j - l_0) / T) the draw moves down iff
   C_{j-1} e^{eps/T} (1-u) >= u (S - C_{j-1}) e^{-eps/T}, up likewise), the
   top-k membership boundary (the k-th vs the (k+1)-th logit) and the order
   of the drawn candidate's neighbours;
3. the same GEMV bound evaluated on that draw's head rows, eps_gemv =
   2e-6 * max_i sum_k |W_ik x_k| + 1e-6 over the candidates.

Verdict: "fp near-tie" if eps_flip <= eps_gemv (the head's own rounding can
flip it), "fp near-tie (carried)" if eps_flip <= CARRY * eps_gemv (x itself
carries the rounding of the 28 + 5 layers before it, each within its own
bound; CARRY = 16), otherwise "bug": no rounding-sized difference of the
logits can produce a different id there, so the GPU's logits were wrong.
"""
import numpy as np

CARRY = 16.0


def _u(bits):
    """orc_rand_uniform / the reference's xorshift over the float bits (K.c:384-393)"""
    s = int(bits) & 0xFFFFFFFF
    s ^= (s << 13) & 0xFFFFFFFF
    s ^= s >> 17
    s ^= (s << 5) & 0xFFFFFFFF
    return np.float32(s & 0x7FFFFFFF) / np.float32(0x7FFFFFFF)


def flip_distance(logits, top_k, top_p, temperature, rng_bits):
    """The drawn id of K.c:407-484's top-k path and the smallest raw-logit
    perturbation that would change it (float64 analysis of the float32 draw).
    Returns dict(result, rank, eps_flip, eps_down, eps_up, eps_topk, eps_order,
    candidates = the sorted candidate ids)."""
    lg = np.asarray(logits, np.float32)
    n = lg.shape[0]
    T = np.float32(temperature if temperature > 0 else 1e-5)
    if not (top_p >= 1.0 and 0 < top_k < n):
        raise ValueError("flip_distance covers the top-k path (top_p 1, 0 < top_k < vocab)")
    v = lg / T
    order = np.lexsort((np.arange(n), -v.astype(np.float64)))   # value desc, index asc
    k = min(top_k, n)
    cand = order[:k]
    p = np.exp((v[cand] - v[cand[0]]).astype(np.float32)).astype(np.float32)
    c32 = np.cumsum(p, dtype=np.float32)                # sequential fp32 sums, as the draw
    u = float(_u(rng_bits))
    r = np.float32(u) * c32[-1]
    j = int(np.argmax(c32 >= r))
    # exact-math boundaries (float64) in raw logit units
    w = np.exp((lg[cand].astype(np.float64) - float(lg[cand[0]])) / float(T))
    C = np.cumsum(w)
    S = C[-1]
    inf = float("inf")
    eps_down = inf if j == 0 else 0.5 * float(T) * np.log(u * (S - C[j - 1]) / ((1 - u) * C[j - 1]))
    eps_up = inf if j == k - 1 or u == 0 else 0.5 * float(T) * np.log((1 - u) * C[j] / (u * (S - C[j])))
    eps_topk = inf if k >= n else 0.5 * float(lg[order[k - 1]] - lg[order[k]])
    nb = [x for x in (j - 1, j + 1) if 0 <= x < k]
    eps_order = min([0.5 * abs(float(lg[cand[j]] - lg[cand[x]])) for x in nb], default=inf)
    eps = min(max(eps_down, 0.0), max(eps_up, 0.0), eps_topk, eps_order)
    return dict(result=int(cand[j]), rank=j, eps_flip=eps, eps_down=eps_down, eps_up=eps_up, eps_topk=eps_topk,
                eps_order=eps_order, u=u, candidates=[int(x) for x in cand])


def _bf16_rows(arr, rows):
    a = np.asarray(arr[rows])
    if a.dtype == np.uint16:
        a = (a.astype(np.uint32) << 16).view(np.float32)
    return a.astype(np.float64)


def gemv_bound(tensors, group, x, rows):
    """2e-6 * sum_k |W_ik x_k| + 1e-6 for the head rows `rows` of draw group
    `group` (0: talker.codec_head, g: code_predictor.lm_head.{g-1})"""
    name = "talker.codec_head.weight" if group == 0 else f"talker.code_predictor.lm_head.{group - 1}.weight"
    W = _bf16_rows(tensors[name][1], np.asarray(rows))
    return 2e-6 * np.abs(W * np.asarray(x, np.float64)[None, :]).sum(axis=1) + 1e-6


def classify(oracle, ids, spk, lang, frame, group, params, got=None):
    """Verdict on the first divergence at (frame, group) of utterance `ids`
    generated with `params` (the oracle's keyword parameters).  got: the id the
    GPU drew there (reported only)."""
    tr = oracle.trace_draw(ids, spk, lang, frame, group, **params)
    if tr is None:
        return dict(verdict="unclassified", why="the reference stopped before this draw")
    if group == 0:
        tk, tp, tt = params.get("top_k", 50), params.get("top_p", 1.0), params.get("temperature", 0.9)
    else:
        tk, tp, tt = params.get("st_top_k", 50), params.get("st_top_p", 1.0), params.get("st_temperature", 0.9)
    try:
        fd = flip_distance(tr["logits"], tk, tp, tt, tr["rng_bits"])
    except ValueError as e:
        return dict(verdict="unclassified", why=str(e))
    if fd["result"] != tr["result"]:
        # (numpy's float32 exp vs glibc expf: the draw is a tie at the draw's own rounding)
        fd.update(eps_flip=0.0)
    rows = fd["candidates"] + ([got] if got is not None and got not in fd["candidates"] else [])
    eg = float(gemv_bound(oracle.tensors, group, tr["x"], rows).max())
    ratio = fd["eps_flip"] / eg
    verdict = "fp near-tie" if ratio <= 1.0 else "fp near-tie (carried)" if ratio <= CARRY else "bug"
    return dict(verdict=verdict, frame=int(frame), group=int(group), reference=tr["result"], got=got,
                eps_flip=fd["eps_flip"], eps_gemv=eg, ratio=ratio, rank=fd["rank"], eps_down=fd["eps_down"],
                eps_up=fd["eps_up"], eps_topk=fd["eps_topk"], eps_order=fd["eps_order"], u=fd["u"])


def describe(c):
    if c.get("verdict") == "unclassified":
        return f"unclassified ({c.get('why')})"
    return (f"{c['verdict']}: the reference's draw (frame {c['frame']}, group {c['group']}, id {c['reference']}, "
            f"GPU {c['got']}) flips under a logit change of {c['eps_flip']:.3g}; the head GEMV's rounding bound "
            f"there is {c['eps_gemv']:.3g} (ratio {c['ratio']:.3g}; down {c['eps_down']:.3g}, up {c['eps_up']:.3g}, "
            f"top-k {c['eps_topk']:.3g}, order {c['eps_order']:.3g})")
