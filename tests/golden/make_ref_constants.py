"""Extract the reference's own numeric constants into tests/golden/ref_constants.json.

Reads /root/reference/CpGIslandFinder.java AS TEXT (it is never compiled or run: no JDK
here) and records, with the line each value sits on:
  * initialP / transitionP / emissionP (:155-173) — the decimal literals as written and the
    IEEE binary64 value each denotes (Python's float() and javac both round a decimal
    literal correctly to nearest, so the hex is the bits the JVM holds);
  * the training / decode chunk sizes (0x10000 at :130-131, 0x100000 at :230, :256-257);
  * the island filter thresholds (cg > 0.5, oe > 0.6 at :285);
  * the Baum-Welch configuration strings (:92-98) and the hidden / emitted state maps
    (:182-194).
The fixture is data (values + line numbers), not reference source.  tests/test_ref_constants.py
checks the library's cpg_initial_model, cpg.h's chunk constants, both oracles and the
island filter against it.  Re-run only in a container holding /root/reference.
"""
import json
import os
import re
import sys

SRC = "/root/reference/CpGIslandFinder.java"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref_constants.json")


def line_of(text, pos):
    return text.count("\n", 0, pos) + 1


def parse_array(text, name):
    """`double[] name = {...};` or `double[][] name = {{...}, ...};` → (rows, first line)."""
    m = re.search(r"double\s*(\[\])+\s*" + re.escape(name) + r"\s*=\s*\{", text)
    if not m:
        raise SystemExit(f"{name} not found in {SRC}")
    i, depth = m.end() - 1, 0
    for j in range(i, len(text)):
        depth += {"{": 1, "}": -1}.get(text[j], 0)
        if depth == 0:
            body = text[i:j + 1]
            break
    rows = re.findall(r"\{([^{}]*)\}", body) if body.count("{") > 1 else [body[1:-1]]
    lits = [[t.strip() for t in r.split(",") if t.strip()] for r in rows]
    return lits, line_of(text, m.start()), line_of(text, i + len(body))


def main():
    with open(SRC) as f:
        text = f.read()
    out = {"source": "CpGIslandFinder.java (read as text by tests/golden/make_ref_constants.py)"}
    for name in ("initialP", "transitionP", "emissionP"):
        lits, l0, l1 = parse_array(text, name)
        vals = [[float(x) for x in r] for r in lits]
        out[name] = {"lines": [l0, l1], "literals": lits if len(lits) > 1 else lits[0],
                     "hex": ([[v.hex() for v in r] for r in vals] if len(lits) > 1
                             else [v.hex() for v in vals[0]])}
    chunks = {}
    for name, pat in (("train_chunk", r"count\s*%\s*(0x[0-9a-fA-F]+)\s*==\s*0\)\)\s*\{\s*Vector"),
                      ("decode_chunk", r"count\s*%\s*(0x[0-9a-fA-F]+)\s*==\s*0\)\)\s*\{\s*for")):
        m = re.search(pat, text)
        chunks[name] = {"literal": m.group(1), "value": int(m.group(1), 16),
                        "line": line_of(text, m.start())}
    m = re.search(r"new\s+DenseVector\((0x[0-9a-fA-F]+)\)", text)
    chunks["train_vector_len"] = {"literal": m.group(1), "value": int(m.group(1), 16),
                                  "line": line_of(text, m.start())}
    m = re.search(r"new\s+int\[(0x[0-9a-fA-F]+)\]", text)
    chunks["decode_array_len"] = {"literal": m.group(1), "value": int(m.group(1), 16),
                                  "line": line_of(text, m.start())}
    out["chunks"] = chunks
    m = re.search(r"\(cgcontent\s*>\s*([0-9.]+)\)\s*&&\s*\(oeratio\s*>\s*([0-9.]+)\)", text)
    out["island_filter"] = {"cg_gt": {"literal": m.group(1), "hex": float(m.group(1)).hex()},
                            "oe_gt": {"literal": m.group(2), "hex": float(m.group(2)).hex()},
                            "line": line_of(text, m.start()),
                            "length_filter_commented_out":
                                "/*(islandLen > 200) && */" in text}
    conf = {}
    for key, val in re.findall(r"conf\.set\(BaumWelchConfigKeys\.(\w+),\s*\"([^\"]*)\"\)", text):
        conf[key] = val
    out["bw_conf"] = conf
    hidden = re.findall(r"hiddenMap\.put\(new Text\(\"([^\"]+)\"\),\s*new IntWritable\((\d+)\)\)", text)
    emitted = re.findall(r"emittedMap\.put\(new Text\(\"([^\"]+)\"\),\s*new IntWritable\((\d+)\)\)", text)
    out["hidden_states"] = {n: int(i) for n, i in hidden}
    out["emitted_symbols"] = {n: int(i) for n, i in emitted}
    # the symbol map of both readers (:114-123, :240-249)
    sym = {}
    for ch, v in re.findall(r"\(chr == '(\w)'\)[^\n]*\n\s*val = (\d)", text):
        sym[ch] = int(v)
    for ch, v in re.findall(r"\|\| \(chr == '(\w)'\)\)\s*\n\s*val = (\d)", text):
        sym[ch] = int(v)
    out["symbol_map"] = sym
    m = re.search(r"String\.format\(\"([^\"]+)\"", text)
    out["island_format"] = {"format": m.group(1), "line": line_of(text, m.start())}
    out["main_args"] = re.findall(r"String (\w+) = args\[(\d)\];", text) + \
        re.findall(r"int (\w+) = Integer\.parseInt\(args\[(\d)\]\);", text)
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print(f"wrote {OUT}")


if __name__ == "__main__":
    sys.exit(main())
