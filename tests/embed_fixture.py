"""Deterministic stand-ins for the embedding half's models (test infrastructure): a tiny seeded encoder,
a word-hash tokenizer and an echoing LLM. Used by tests/golden/make_embed_golden.py to run the
REFERENCE's BatchProcessor._process_batch (batch_processor.py:74-125) and by tests/test_embed_pin.py to
run ours on the same inputs. Real e5 / Qwen weights are not available offline (parity for them stays
unpinned); what these pin is the path around the models: prefix, tokenizer call, device moves, the
pad-inclusive mean over positions, the hand-off to batch_retrieve, prompt assembly and result storage.

The encoder's weights come from a NumPy PCG64 stream (seed below), so they are the same on every host
without a weight file."""
import zlib

import numpy as np

H = 1024          # the corpus dimension (short_facts / SQuAD embeddings)
VOCAB = 2048
MAX_LEN = 24      # short enough that some questions are truncated
SEED = 20260


def encoder_weights():
    rng = np.random.default_rng(SEED)
    return {"tok": (rng.standard_normal((VOCAB, H)) * 0.05).astype(np.float32),
            "pos": (rng.standard_normal((MAX_LEN, H)) * 0.02).astype(np.float32),
            "w1": (rng.standard_normal((H, 128)) / np.sqrt(H)).astype(np.float32),
            "w2": (rng.standard_normal((128, H)) / np.sqrt(128)).astype(np.float32)}


def make_encoder():
    import torch

    class TinyEncoder(torch.nn.Module):
        def __init__(self):
            super().__init__()
            w = encoder_weights()
            for name, v in w.items():
                self.register_buffer(name, torch.from_numpy(v))

        def forward(self, input_ids, attention_mask):
            L = input_ids.shape[1]
            x = self.tok[input_ids] + self.pos[:L]
            x = x * (0.5 + attention_mask[..., None].to(x.dtype))      # pads carry a different weight
            h = x + torch.tanh(x @ self.w1) @ self.w2
            h = torch.nn.functional.layer_norm(h, (H,))

            class Out:
                last_hidden_state = h
            return Out()

    return TinyEncoder().eval()


class HashTokenizer:
    """<s>=0, <pad>=1, </s>=2, words -> 5 + crc32 % (VOCAB - 5); right padding to the longest; truncation to
    MAX_LEN (keeping </s>), as an HF tokenizer called with padding=True, truncation=True."""

    def __call__(self, texts, padding=True, truncation=True, return_tensors="pt"):
        import torch
        ids = []
        for t in texts:
            body = [5 + zlib.crc32(w.encode()) % (VOCAB - 5) for w in t.split()]
            seq = [0] + body + [2]
            if truncation and len(seq) > MAX_LEN:
                seq = seq[:MAX_LEN - 1] + [2]
            ids.append(seq)
        L = max(len(s) for s in ids)
        return {"input_ids": torch.tensor([s + [1] * (L - len(s)) for s in ids]),
                "attention_mask": torch.tensor([[1] * len(s) + [0] * (L - len(s)) for s in ids])}


class EchoLLM:
    """Returns "<answer to: prompt>" per prompt and records the prompts."""

    def __init__(self):
        self.prompts = []

    def __call__(self, texts, max_new_tokens=10, do_sample=True, batch_size=None):
        texts = [str(t) for t in texts]
        self.prompts.append(texts)
        return [f"<answer to: {t}>" for t in texts]


# the request batches both sides run: (queries index range or list, ks)
def batches(queries):
    return [
        [{"id": f"a{i}", "query": queries[i], "k": 2} for i in range(32)],
        [{"id": f"b{i}", "query": queries[40 + i], "k": k} for i, k in enumerate([1, 3, 5, 0, 2, 10, 4])],
        [{"id": "c0", "query": queries[99], "k": 100}, {"id": "c1", "query": queries[50], "k": 7}],
    ]
