"""Stage-1 text analysis (bm25s.tokenize + PyStemmer "english", which the
reference calls at local_rag_complete.py:851-855 and 939-943).

The Snowball English stemmer (csrc/text_en.cpp) is pinned by word/stem pairs
restated from the Snowball project's published English description and sample
vocabulary (snowballstem.org, algorithms/english): the "consign..." and
"knack..." runs of its sample output, the special-word lists (exception 1 and
2), and the rules' worked examples.  PyStemmer itself is not installed, so
parity beyond these words is unpinned.  The tokenizer follows bm25s.tokenize:
lower-case, (?u)\\b\\w\\w+\\b, stopwords before stemming, vocabulary stemmed once.
"""
import numpy as np
import pytest

from hybrid_rag_colbertv2_amd.bm25 import STOPWORDS_EN, HostBM25, Stemmer, Tokenized, tokenize

SAMPLE = {  # published sample vocabulary -> output
    "consign": "consign", "consigned": "consign", "consigning": "consign", "consignment": "consign",
    "consist": "consist", "consisted": "consist", "consistency": "consist", "consistent": "consist",
    "consistently": "consist", "consisting": "consist", "consists": "consist", "consolation": "consol",
    "consolations": "consol", "consolatory": "consolatori", "console": "consol", "consoled": "consol",
    "consoles": "consol", "consolidate": "consolid", "consolidated": "consolid", "consolidating": "consolid",
    "consoling": "consol", "consolingly": "consol", "consols": "consol", "consonant": "conson",
    "consort": "consort", "consorted": "consort", "consorting": "consort", "conspicuous": "conspicu",
    "conspicuously": "conspicu", "conspiracy": "conspiraci", "conspirator": "conspir",
    "conspirators": "conspir", "conspire": "conspir", "conspired": "conspir", "conspiring": "conspir",
    "constable": "constabl", "constables": "constabl", "constance": "constanc", "constancy": "constanc",
    "constant": "constant",
    "knack": "knack", "knackeries": "knackeri", "knacks": "knack", "knag": "knag", "knave": "knave",
    "knaves": "knave", "knavish": "knavish", "kneaded": "knead", "kneading": "knead", "knee": "knee",
    "kneel": "kneel", "kneeled": "kneel", "kneeling": "kneel", "kneels": "kneel", "knees": "knee",
    "knell": "knell", "knelt": "knelt", "knew": "knew", "knick": "knick", "knif": "knif", "knife": "knife",
    "knight": "knight", "knightly": "knight", "knights": "knight", "knit": "knit", "knits": "knit",
    "knitted": "knit", "knitting": "knit", "knives": "knive", "knob": "knob", "knobs": "knob",
    "knock": "knock", "knocked": "knock", "knocker": "knocker", "knockers": "knocker", "knocking": "knock",
    "knocks": "knock", "knopp": "knopp", "knot": "knot", "knots": "knot",
}
EXCEPTIONS = {  # exception list 1 (whole words), list 2 (after step 1a), invariants
    "skis": "ski", "skies": "sky", "dying": "die", "lying": "lie", "tying": "tie", "idly": "idl",
    "gently": "gentl", "ugly": "ugli", "early": "earli", "only": "onli", "singly": "singl", "sky": "sky",
    "news": "news", "howe": "howe", "atlas": "atlas", "cosmos": "cosmos", "bias": "bias", "andes": "andes",
    "inning": "inning", "innings": "inning", "outing": "outing", "outings": "outing", "canning": "canning",
    "herring": "herring", "herrings": "herring", "earring": "earring", "proceed": "proceed",
    "proceeds": "proceed", "exceed": "exceed", "succeed": "succeed",
}
RULES = {  # the description's worked examples, rule by rule
    # step 1a
    "caresses": "caress", "ties": "tie", "cries": "cri", "gas": "gas", "this": "this", "gaps": "gap",
    "kiwis": "kiwi", "us": "us", "ss": "ss",
    # step 1b
    "feed": "feed", "agreed": "agre", "luxuriated": "luxuri", "hoped": "hope", "hopping": "hop",
    "sized": "size", "filing": "file", "bled": "bled", "troubled": "troubl",
    # step 1c
    "cry": "cri", "by": "by", "say": "say",
    # regions: gener-, commun-, arsen- prefixes
    "generously": "generous", "generate": "generat", "communism": "communism", "communication": "communic",
    "arsenal": "arsenal",
    # steps 2-5
    "relational": "relat", "conditional": "condit", "rational": "ration", "valenci": "valenc",
    "digitizer": "digit", "operator": "oper", "feudalism": "feudal", "decisiveness": "decis",
    "hopefulness": "hope", "callousness": "callous", "formaliti": "formal", "sensitiviti": "sensit",
    "sensibiliti": "sensibl", "triplicate": "triplic", "formative": "format", "formalize": "formal",
    "electriciti": "electr", "electrical": "electr", "hopeful": "hope", "goodness": "good",
    "revival": "reviv", "allowance": "allow", "inference": "infer", "airliner": "airlin",
    "gyroscopic": "gyroscop", "adjustable": "adjust", "defensible": "defens", "irritant": "irrit",
    "replacement": "replac", "adjustment": "adjust", "dependent": "depend", "adoption": "adopt",
    "communism2": "communism2", "activate": "activ", "angulariti": "angular", "homologous": "homolog",
    "effective": "effect", "bowdlerize": "bowdler", "controll": "control", "roll": "roll",
    "yes": "yes", "yield": "yield", "sayings": "say", "playing": "play",
}


def test_stemmer_published_vocabulary():
    st = Stemmer("english")
    for table in (SAMPLE, EXCEPTIONS):
        words = list(table)
        got = st.stemWords(words)
        bad = [(w, g, table[w]) for w, g in zip(words, got) if g != table[w]]
        assert not bad, bad


def test_stemmer_rule_examples():
    st = Stemmer("english")
    bad = [(w, st.stemWord(w), s) for w, s in RULES.items() if st.stemWord(w) != s]
    assert not bad, bad


def test_stemmer_edges():
    st = Stemmer("english")
    assert st.stemWords([]) == []
    assert st.stemWords(["a", "is", "", "x1", "über", "naïve", "café"]) == ["a", "is", "", "x1", "über", "naïv", "café"]
    assert st.stemWord("'tis") == "tis" and st.stemWord("dog's") == "dog"
    with pytest.raises(ValueError):
        Stemmer("french")


def test_tokenize_follows_bm25s():
    st = Stemmer("english")
    tk = tokenize(["The Cats are running!", "a I x", "Running cats: 42 e-mails"], stopwords="en", stemmer=st)
    assert isinstance(tk, Tokenized)
    inv = {v: k for k, v in tk.vocab.items()}
    rows = [[inv[t] for t in r] for r in tk.ids]
    # "the", "are", "a" are stopwords; one-letter tokens never match \w\w+; stems shared
    assert rows == [["cat", "run"], [], ["run", "cat", "42", "mail"]]
    assert tokenize("a is it", stopwords="en", stemmer=st).ids == [[]]     # one (empty) row per text
    assert set(STOPWORDS_EN) >= {"the", "and", "is", "it", "with"} and len(STOPWORDS_EN) == 33
    assert tokenize(["Cats"], stopwords=None, stemmer=None, return_ids=False) == [["cats"]]
    with pytest.raises(ValueError):
        tokenize(["x"], stopwords="fr")


def test_hostbm25_stopword_only_query_and_unknown_terms():
    corpus = ["The cat sat on the mat", "Dogs chase cats", "A bird in the hand", "Cats and dogs and cats"]
    bm = HostBM25()
    bm.index(tokenize(corpus, stopwords="en", stemmer=Stemmer("english")))
    for q in ("is it?", "?", "", "zebra unicorn"):
        ids, sc = bm.retrieve(tokenize(q, stopwords="en", stemmer=Stemmer("english")), k=3)
        assert ids.shape == (1, 3) and (sc == 0).all() and ids[0].tolist() == [0, 1, 2]
    ids, sc = bm.retrieve(tokenize("cats", stopwords="en", stemmer=Stemmer("english")), k=3)
    assert ids[0][0] == 3 and sc[0][0] > sc[0][1] > 0
    # repeated query words count once per occurrence (bm25s sums every query token)
    _, s1 = bm.retrieve(tokenize("dog", stopwords="en", stemmer=Stemmer("english")), k=1)
    _, s2 = bm.retrieve(tokenize("dog dogs", stopwords="en", stemmer=Stemmer("english")), k=1)
    assert np.isclose(s2[0][0], 2 * s1[0][0])


def test_hybrid_bm25_stage_stopword_query():
    """HybridRetriever._bm25_search (LRC:937-950) on a stopword-only query: k
    results (zero scores), no IndexError."""
    from hybrid_rag_colbertv2_amd.config import RAGConfig
    from hybrid_rag_colbertv2_amd.encoder import FakeEncoder
    from hybrid_rag_colbertv2_amd.hybrid import DualIndexer, HybridRetriever
    cfg = RAGConfig()
    ix = DualIndexer.__new__(DualIndexer)
    ix.config, ix.colbert_retriever = cfg, None
    ix.bm25_retriever = HostBM25()
    ix.bm25_retriever.index(tokenize(["cats and dogs", "a mat", "the bird"], stopwords="en",
                                     stemmer=Stemmer("english")))
    hr = HybridRetriever(cfg, ix, verbose=False)
    res = hr._bm25_search("is it?", k=2)
    assert [r["chunk_id"] for r in res] == [0, 1] and all(r["score"] == 0.0 for r in res)
    assert hr._bm25_search("dog", k=1)[0]["chunk_id"] == 0
    assert FakeEncoder is not None
