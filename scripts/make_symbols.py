"""Writes configs/symbols.json: the reference's phoneme/character symbol table
(text/symbols.py:23-33, ids = list positions), the vocabulary Dataset maps phone strings
through (dataset.py:21,45).  Run in the build container, where /root/reference exists; only
the resulting table (data) is committed."""
import json
import os
import sys
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, "/root/reference")
sys.dont_write_bytecode = True
for n in ("unidecode", "inflect"):  # import-time only (text/cleaners.py, text/numbers.py)
    sys.modules.setdefault(n, types.ModuleType(n))
sys.modules["unidecode"].unidecode = lambda s: s
sys.modules["inflect"].engine = lambda: None
from text.symbols import symbols  # noqa: E402

out = os.path.join(REPO, "mid-attribute-speaker-generation_amd", "configs", "symbols.json")
with open(out, "w", encoding="utf-8") as f:
    json.dump(symbols, f, ensure_ascii=False)
print(f"{len(symbols)} symbols -> {out}")
