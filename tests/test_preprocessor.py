"""Parity ports of reference tests/preprocessor_test.go + Go-semantics
oracle checks (the oracle is the bit-exact target of the HIP kernels)."""
import pytest

from llm_message_queue_amd.gateway.workload import HIGH_KW, NEUTRAL, REALTIME_KW, Workload
from llm_message_queue_amd.models.message import Message
from llm_message_queue_amd.preprocess import oracle
from llm_message_queue_amd.preprocess.preprocessor import Preprocessor


@pytest.fixture
def pre():
    return Preprocessor(use_gpu=False)


def test_content_based_priority(pre):
    m = pre.process_message(Message(content="This is an urgent request", priority=0))
    assert m.priority == 2


def test_user_priority_override(pre):
    m = pre.process_message(Message(content="hello", metadata={"user_priority": "high"}))
    assert m.priority == 2 and m.metadata["priority_reason"] == "user_override"


def test_respect_explicit_priority(pre):
    m = pre.process_message(Message(content="urgent", priority=1))
    assert m.priority == 1 and "analyzed" not in m.metadata


def test_metadata_based_priority(pre):
    m = pre.process_message(Message(content="hello", metadata={"source": "api"}))
    assert m.metadata["source"] == "api" and m.metadata["analyzed"] is True


def test_custom_keyword_patterns(pre):
    m = pre.process_message(Message(content="I need this right now, it's immediate"))
    assert m.priority == 1 and m.metadata["priority_reason"] == "content_keywords"


def test_content_analysis(pre):
    m = pre.process_message(Message(content="Is this a good question?"))
    assert m.metadata["contains_question"] == "true"
    assert "sentiment" in m.metadata and m.metadata["sentiment"] == "positive"


def test_user_default_and_queue_name(pre):
    pre.set_user_priority("alice", 4)
    m = pre.process_message(Message(content="urgent!", user_id="alice"))
    assert m.priority == 4 and m.metadata["priority_reason"] == "user_default" and m.queue_name == "low"


def test_empty_content_metadata_priority(pre):
    m = pre.process_message(Message(content="", metadata={"priority": "LOW"}))
    assert m.priority == 4 and "word_count" not in m.metadata


def test_add_keyword_pattern_and_default(pre):
    pre.add_keyword_pattern(4, "(?i)whenever")
    assert pre.process_message(Message(content="Whenever you can")).priority == 4
    pre.set_default_priority(2)
    assert pre.process_message(Message(content="plain")).priority == 2
    assert pre.get_keyword_patterns(4) == ["(?i)whenever"]
    with pytest.raises(Exception):
        pre.add_keyword_pattern(1, "(unclosed")


def test_analyze_message_content(pre):
    r = pre.analyze_message_content("what a terrible awful day")
    assert r == {"word_count": 5, "sentiment": "negative", "is_question": True}


# ---------------------------------------------------------------- Go semantics
def test_fields_go_whitespace():
    assert oracle.go_fields("a\x1cb c") == ["a\x1cb", "c"]          # U+001C is not a Go space
    assert oracle.go_fields("a b　c d") == ["a", "b", "c", "d"]
    assert oracle.go_fields("  ") == []


def test_lower_and_fold_specials():
    assert oracle.go_lower("İK") == "ik"
    assert oracle.keyword_scores("aſap", oracle.default_patterns())[1] == 1
    assert oracle.content_analysis("GOOD")[1] == "positive"
    assert oracle.content_analysis("good!")[1] == "neutral"          # punctuation is not stripped


def test_question_substring_semantics():
    assert oracle.is_question("somewhat odd")                          # "what " substring
    assert not oracle.is_question("question? ")                        # HasSuffix, no trim
    assert oracle.is_question("x?")


def test_non_overlapping_counts_and_ties():
    pats = {1: [oracle.compile_pattern("aa")], 2: [oracle.compile_pattern("(?i)b")]}
    assert oracle.keyword_scores("aaaa", pats)[1] == 2
    assert oracle.keyword_scores("aaa", pats)[1] == 1
    assert oracle.pick_priority({1: 2, 2: 2}, 3) == 1                  # deterministic tie (D17)
    assert oracle.pick_priority({1: 0, 2: 0}, 3) == 3


def test_compile_pattern_kinds():
    assert isinstance(oracle.compile_pattern("(?i)urgent"), oracle.LiteralPattern)
    assert isinstance(oracle.compile_pattern("right\\ now"), oracle.LiteralPattern)
    assert isinstance(oracle.compile_pattern("urg.nt"), oracle.RegexPattern)


def test_workload_vocabulary_is_keyword_free():
    pats = oracle.default_patterns()
    text = " ".join(NEUTRAL)
    assert all(v == 0 for v in oracle.keyword_scores(text, pats).values())
    for kw in REALTIME_KW:
        assert oracle.keyword_scores(kw, pats)[1] >= 1
    for kw in HIGH_KW:
        assert oracle.keyword_scores(kw, pats)[2] >= 1


def test_workload_mix_through_preprocessor(pre):
    msgs = Workload(seed=3).make(2000)
    pre.process_batch(msgs, use_gpu=False)
    counts = [0, 0, 0, 0]
    for m in msgs:
        counts[m.priority - 1] += 1
    frac = [c / 2000 for c in counts]
    for f, want in zip(frac, (0.1, 0.3, 0.4, 0.2)):
        assert abs(f - want) < 0.04


def test_token_hashes():
    h = oracle.token_hashes("Hello  WORLD x" + "y" * 40, 8)
    assert h[0] == oracle.fnv1a32(b"hello") and h[1] == oracle.fnv1a32(b"world")
    assert h[2] == oracle.fnv1a32(b"x" + b"y" * 31)


@pytest.mark.parametrize("B", [0, 1, 17, 40, 41, 300])
def test_kernel_side_decisions_match_score_argmax(B):
    """TextResult.decide's fast paths (per-row for small batches, numpy for
    large) read the slot / code words text_analyze writes into stats columns
    6-7; they must equal the score-argmax decision of the general path."""
    import numpy as np
    from llm_message_queue_amd.ops.text import TextResult
    rng = np.random.default_rng(B)
    st = np.zeros((B, 16), dtype=np.int32)
    st[:, 0] = rng.integers(0, 50, B)                    # words
    st[:, 1:3] = rng.integers(0, 3, (B, 2))             # pos, neg
    st[:, 3] = rng.integers(0, 2, B)                     # question
    st[:, 4] = rng.integers(0, 2, B)                     # fold flag
    st[:, 5] = rng.integers(0, 60, B)                    # ntok
    st[:, 8:12] = rng.integers(0, 3, (B, 4))            # 4 keyword slots, ties common
    for r in st:                                         # what the kernel writes
        sc = r[8:16]
        r[6] = int(np.argmax(sc)) if sc.max() > 0 else -1
        r[7] = (1 if r[1] > r[2] else 2 if r[2] > r[1] else 0) | (4 if r[3] else 0) | (8 if r[4] else 0)
    ph = np.zeros((B, 32), dtype=np.uint32)
    fast = TextResult(st, None, 0.0, False, [0, 1, 2, 3], None, None, None, 128, ph).decide(2)
    slow = TextResult(st, None, 0.0, False, [0, 1, 2, 3], np.zeros((B, 8), dtype=np.int64), None, None, 128,
                      ph).decide(2)
    for k in ("priority", "sentiment", "question", "word_count", "fallback", "ntok"):
        assert list(fast[k]) == list(slow[k]), k


def test_export_load_state_round_trip():
    """The admin state a multi-rank job copies from rank 0 to every rank
    (gateway.app.sync_preprocessor): rules, user defaults, default priority."""
    a, b = Preprocessor(use_gpu=False), Preprocessor(use_gpu=False)
    a.add_keyword_pattern(1, "(?i)zebra")
    a.remove_keyword_pattern(2, "(?i)soon")
    a.set_user_priority("alice", 4)
    a.set_default_priority(2)
    b.load_state(a.export_state())
    assert b.all_patterns() == a.all_patterns() and b.user_priorities() == {"alice": 4}
    assert b.default_priority == 2
    assert b.process_message(Message(content="a zebra", user_id="bob")).priority == 1
    assert b.process_message(Message(content="a zebra", user_id="alice")).priority == 4
    assert b.process_message(Message(content="soon", user_id="bob")).priority == 2     # rule gone -> default
    with pytest.raises(Exception):
        b.load_state({"patterns": [[1, ["(unclosed"]]], "user_priorities": {}, "default_priority": 3})
    assert b.all_patterns() == a.all_patterns()                                          # unchanged on error


def test_record_analysis_matches_analyze_message_content():
    """Behind the C++ front door the ranks preprocess raw requests, so they
    record metadata["analysis"] (AnalyzeMessageContent as Go's json.Marshal
    emits it, `api/handlers.go:181-191`) for every message -- explicit
    priority and empty content included -- on the batch paths too."""
    import json as _json
    texts = ["Is this a good question?", "urgent: bad bad service", "", "KELVIN K what now", "plain words",
             "happy", "terrible?"]
    for native in (True, False):
        pre = Preprocessor(use_gpu=False)
        pre.record_analysis = True
        if not native:
            pre.cfg.native_cpu = False
        msgs = [Message(content=t, priority=(4 if i % 3 == 1 else 0)) for i, t in enumerate(texts)]
        pre.process_batch(msgs, use_gpu=False, prompt_cap=8)
        for m in msgs:
            want = pre.analyze_message_content(m.content)
            got = m.metadata["analysis"]
            assert _json.loads(got) == want, (native, m.content, got)
            assert list(_json.loads(got)) == ["is_question", "sentiment", "word_count"]   # Go map order
    off = Preprocessor(use_gpu=False)
    ms = [Message(content="hello")]
    off.process_batch(ms, use_gpu=False)
    assert "analysis" not in ms[0].metadata
