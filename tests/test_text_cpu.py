"""The CPU twin of the text_analyze kernel (csrc/text/text_cpu.h, module
_textcpu) against the Python oracle of the reference's Go preprocessor
(preprocess/oracle.py): word counts, sentiment, question, keyword scores
(literal, case-insensitive, self-overlapping, non-ASCII patterns; regex
patterns scored on the host), fold-special fallback flags and token hashes --
the same checks tests/test_gpu_kernels.py runs on the GPU kernel.  Plus the
Preprocessor's CPU batch path == its per-message oracle path.
"""
import numpy as np
import pytest

from llm_message_queue_amd.preprocess import oracle
from text_cases import ADVERSARIAL, _random_texts


def _pipe(L=64):
    from llm_message_queue_amd.ops.text import CpuTextPipeline
    from llm_message_queue_amd.utils.config import PreprocessorConfig
    return CpuTextPipeline(PreprocessorConfig(max_tokens=L))


def _check(texts, patterns=None, L=64):
    pats = patterns or oracle.default_patterns()
    res = _pipe(L).run(texts, pats, prompt_cap=L)
    for j, t in enumerate(texts):
        t = oracle.sanitize(t)
        wc, sent, q = oracle.content_analysis(t)
        pos, neg = oracle.sentiment_counts(t)
        fold = any(c in oracle.FOLD_SPECIAL for c in t)
        assert bool(res.fallback[j]) == fold, (repr(t), res.stats[j])
        assert res.stats[j, 0] == wc, (repr(t), res.stats[j, 0], wc)
        assert bool(res.question[j]) == q, repr(t)
        if not fold:
            assert (res.stats[j, 1], res.stats[j, 2]) == (pos, neg), (repr(t), res.stats[j])
            assert res.scores(j) == oracle.keyword_scores(t, pats), (repr(t), res.scores(j))
        th = oracle.token_hashes(t, L)
        assert res.stats[j, 5] == len(th)
        assert list(res.prompt_hashes[j, :len(th)]) == th, repr(t)


def test_cpu_twin_adversarial():
    _check(ADVERSARIAL)


def test_cpu_twin_random():
    _check(_random_texts(1500, seed=3))


def test_cpu_twin_custom_patterns():
    pats = oracle.default_patterns()
    pats.setdefault(4, []).append(oracle.compile_pattern("(?i)later"))
    pats[2].append(oracle.compile_pattern("aa"))           # self-overlapping (bordered)
    pats[2].append(oracle.compile_pattern("Case"))         # case-sensitive
    pats[1].append(oracle.compile_pattern("紧急"))          # non-ASCII literal
    pats[4].append(oracle.compile_pattern("(?i)l[a-z]+r"))  # regex -> host path
    texts = ["aaaa later LATER Case case", "紧急 紧急紧急", "aaa", "lover later", "CASE"] + _random_texts(200, 9)
    _check(texts, pats)


def test_cpu_twin_decisions_match_score_argmax():
    """Columns 6-7 (best slot, code word) agree with the scores and counts."""
    res = _pipe().run(_random_texts(400, seed=5), oracle.default_patterns())
    st = res.stats
    for r in st:
        sc = r[8:16]
        assert r[6] == (int(np.argmax(sc)) if sc.max() > 0 else -1)
        assert r[7] == ((1 if r[1] > r[2] else 2 if r[2] > r[1] else 0) | (4 if r[3] else 0) | (8 if r[4] else 0))


@pytest.mark.parametrize("prompt_cap", [0, 32])
def test_preprocessor_cpu_batch_matches_per_message_oracle(prompt_cap):
    from llm_message_queue_amd.gateway.workload import Workload
    from llm_message_queue_amd.models.message import Message
    from llm_message_queue_amd.preprocess.preprocessor import Preprocessor
    msgs_a = Workload(seed=7).make(400)
    extra = [("aſap now", 0), ("", 0), ("help", 2), ("x", 3), ("", 5)]
    for c, p in extra:
        msgs_a.append(Message(id="e", content=c, priority=p))
    msgs_b = [m.copy() for m in msgs_a]
    fast = Preprocessor(use_gpu=False)
    assert fast.cpu_pipeline() is not None
    fast.process_batch(msgs_a, use_gpu=False, prompt_cap=prompt_cap)
    from llm_message_queue_amd.utils.config import PreprocessorConfig
    slow = Preprocessor(PreprocessorConfig(native_cpu=False), use_gpu=False)
    slow.process_batch(msgs_b, use_gpu=False, prompt_cap=prompt_cap)
    assert fast.stats["cpu_native_messages"] > 0 and slow.stats["cpu_messages"] > 0
    assert slow.cpu_pipeline() is None
    for a, b in zip(msgs_a, msgs_b):
        assert a.priority == b.priority, (a.content, a.priority, b.priority)
        assert a.metadata == b.metadata, (a.content, a.metadata, b.metadata)
        assert a.queue_name == b.queue_name
        if prompt_cap:                          # None == no tokens (the router gives both a 1-token prompt)
            ids = [lambda x: [] if x is None else [int(v) for v in x]][0]
            assert ids(a.prompt_ids) == ids(b.prompt_ids), a.content
