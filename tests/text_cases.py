"""Shared text cases for the text-analysis tests (GPU kernel and its CPU twin)."""
import random

ADVERSARIAL = [
    "", "?", " ", "URGENT", "urgent urgent", "aſap please", "KELVIN K and İstanbul good",
    "somewhat unclear", "what is this", "WHAT is", "How are you", "who", "who ",
    "good", "GOOD bad", "good! bad", "good bad", "good　happy sad", "tab\tgood\nbad\rterrible",
    "\x1cgood\x1c", "emergency emergency asap immediate right now now", "right  now",
    "critical soon important priority urgent", "prioritySetting", "immediately", "ASAPasap",
    "\xff\xfe invalid?", "é good é", "good\u0085bad", " good ", " why  ",
    "x" * 1000 + " urgent " + "y" * 1000, " ".join(["good"] * 300), "where where where? ",
    "frustrated frustrated happy", "satisfied excellent great happy good", "awful angry",
    "why　 not", "when ", "emergencyemergency", "soonsoon", "a" * 70 + "urgent",
    "日本語 urgent 中文 good", "Ünïcödé ÉMERGENCY",
]

WORDS = ["good", "bad", "urgent", "asap", "what", "how", "why", "soon", "right", "now", "happy",
         "angry", "critical", "emergency", "priority", "terrible", "who", "where", "é", "日本", "Good",
         "URGENT", "Now", "x", "test", "important", "immediate"]
SEPS = [" ", "  ", "\t", "\n", " ", "　", " ", ",", ".", "?", "!", "\u0085", "\x1c"]


def _random_texts(n, seed=0):
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        k = rng.randint(0, 40)
        parts = []
        for _ in range(k):
            parts.append(rng.choice(WORDS))
            parts.append(rng.choice(SEPS))
        s = "".join(parts)
        if rng.random() < 0.2:
            s += "?"
        out.append(s)
    return out
