"""tokenize_patient_details (TP:335-342) on the WordPiece path (MMDX_BERT_VOCAB set).

The reference builds `AutoTokenizer.from_pretrained("bert-base-uncased")` (TP:323), a
BertTokenizerFast: lower-casing, BERT basic tokenisation (whitespace + punctuation split),
greedy longest-match-first WordPiece with "##" continuations and [UNK] for words with no
match, [CLS] ... [SEP], truncation to max_length, padding with [PAD] = id 0.  The real
vocabulary cannot be fetched offline, so this test writes a small vocab.txt and checks the
mmdx tokenizer against an independent pure-Python restatement of that published algorithm
(ids, attention mask, token types, truncation, padding).  The hash-word stand-in used when no
vocab is configured is covered by test_surface_cpu.py::test_tokenize_contract.
"""
import re

import pytest
import torch

import mmdx
from mmdx import training_pipeline as TPL

VOCAB = ["[PAD]", "[unused0]", "[UNK]", "[CLS]", "[SEP]", "[MASK]", ",", ";", ".", "67",
         "m", "f", "54", "no", "smoke", "##r", "smoking", "dy", "##sp", "##nea", "cough",
         "ch", "##f", "history", "asthma", "hyper", "##tension", "##s", "with"]


def _wordpiece_ref(text, vocab, max_len):
    """Greedy longest-match-first WordPiece over BERT basic tokens (uncased)."""
    idx = {t: i for i, t in enumerate(vocab)}
    ids = []
    for word in re.findall(r"\w+|[^\w\s]", text.lower()):
        start, pieces = 0, []
        while start < len(word):
            end, cur = len(word), None
            while start < end:
                sub = word[start:end] if start == 0 else "##" + word[start:end]
                if sub in idx:
                    cur = sub
                    break
                end -= 1
            if cur is None:
                pieces = ["[UNK]"]
                break
            pieces.append(cur)
            start = end
        ids += [idx[p] for p in pieces]
    ids = [idx["[CLS]"]] + ids[: max_len - 2] + [idx["[SEP]"]]
    mask = [1] * len(ids) + [0] * (max_len - len(ids))
    return ids + [idx["[PAD]"]] * (max_len - len(ids)), mask


@pytest.fixture
def wordpiece(tmp_path, monkeypatch):
    pytest.importorskip("tokenizers")
    v = tmp_path / "vocab.txt"
    v.write_text("\n".join(VOCAB) + "\n")
    monkeypatch.setenv("MMDX_BERT_VOCAB", str(v))
    saved = TPL._TOKENIZER[0]
    TPL._TOKENIZER[0] = None
    yield
    TPL._TOKENIZER[0] = saved


@pytest.mark.parametrize("max_len", [96, 8])
def test_wordpiece_path_matches_the_algorithm(wordpiece, max_len):
    texts = ["67M, smoker; dyspnea; CHF history.",
             "54F, no smoking; cough; asthma with hypertension.",
             "unknownword; COUGH"]
    tok = mmdx.tokenize_patient_details(texts, max_len=max_len)
    assert tuple(tok["input_ids"].shape) == (3, max_len)
    for i, t in enumerate(texts):
        ids, mask = _wordpiece_ref(t, VOCAB, max_len)
        assert tok["input_ids"][i].tolist() == ids, t
        assert tok["attention_mask"][i].tolist() == mask, t
    assert (tok["token_type_ids"] == 0).all()
    assert tok["input_ids"].dtype == torch.long


def test_wordpiece_splits_and_unknowns(wordpiece):
    tok = mmdx.tokenize_patient_details(["dyspnea xyz"], max_len=8)
    # [CLS] dy ##sp ##nea [UNK] [SEP] [PAD] [PAD]
    assert tok["input_ids"][0].tolist() == [3, 17, 18, 19, 2, 4, 0, 0]
