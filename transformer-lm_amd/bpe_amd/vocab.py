"""Vocab -- mirror of reference models/tokenizer/vocab.py:1-43 (host-side bookkeeping).

Ids: special tokens in order, then the 256 single bytes, then each added token; a byte string
already present is not added again (vocab.py:28-34).  Membership is a hash set here rather than
the reference's O(V) scan of dict values; the ids produced are the same.
"""
from __future__ import annotations


class Vocab:
    def __init__(self, special_tokens: list[str] = []) -> None:
        self.idx_to_token: dict[int, bytes] = {}
        self._present: set[bytes] = set()
        for token in special_tokens:
            self.add_token(token.encode("utf-8"))
        for i in range(256):
            self.add_token(bytes([i]))
        self.unk_idx: int = 0

    @classmethod
    def from_dict(cls, vocab: dict[int, bytes], special_tokens: list[str] = []) -> "Vocab":
        inst = cls(special_tokens)
        inst.idx_to_token = vocab
        inst._present = set(vocab.values())
        return inst

    def __len__(self) -> int:
        return len(self.idx_to_token)

    def __getitem__(self, idx: int) -> bytes:
        return self.idx_to_token.get(idx, self.idx_to_token[self.unk_idx])

    def add_token(self, token: bytes) -> None:
        if token in self._present:
            return
        self.idx_to_token[len(self.idx_to_token)] = token
        self._present.add(token)

    def get_inv(self) -> dict[bytes, int]:
        return {v: k for k, v in self.idx_to_token.items()}

    def get_idx_to_token(self) -> dict[int, bytes]:
        return self.idx_to_token

    def set_unk_idx(self, unk_idx: int) -> None:
        self.unk_idx = unk_idx
