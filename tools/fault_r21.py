#!/usr/bin/env python3
"""Round-4 counter fault (DESIGN.md §3.5 "Round 6"): static checks of the failing kernel.

Build the round-5-start tree (git 21fc9ac, the tree the fault was bisected on) with -DAGX_SPARSE_SERIAL:
    mkdir -p /tmp/t21 && git archive 21fc9ac akka_amd include | tar -x -C /tmp/t21
    hipcc ... -DAGX_SPARSE_SERIAL -DAGX_VGROUP=7 --save-temps -c /tmp/t21/akka_amd/csrc/agx_apply.hip   (-> ISA .s)
    clang++ -x hip ... --cuda-device-only -S -emit-llvm -o dev.ll ...                                  (-> optimised IR)
then:  python tools/fault_r21.py <isa.s> <dev.ll>
Prints, for k_bucket_apply<true, 1792, false, false, false> (the wide CRDT multi-pass kernel of
test_multipass_grouping[crdt]): its register / spill metadata, every phi with an undef / poison input
in its optimised IR and the def-use chain of each flushed counter (acc[0..4]), and the reaching
definitions (scalar CFG) of the registers added into the counters at the bucket-loop latch."""
import re
import sys

NAME = "_ZN3agxL14k_bucket_applyILb1ELj1792ELb0ELb0ELb0EEEvNS_10BucketArgsE"


def ir_checks(path):
    L = open(path).read().split("\n")
    st = [i for i, l in enumerate(L) if l.startswith("define") and NAME in l][0]
    en = [i for i in range(st, len(L)) if L[i] == "}"][0]
    body = L[st:en + 1]
    defs = {}
    for i, l in enumerate(body):
        m = re.match(r"\s+(%\d+) = (.*)", l)
        if m:
            defs[m.group(1)] = m.group(2)
    undef = [l.strip() for l in body if " phi " in l and ("undef" in l or "poison" in l)]
    print(f"IR: {len(body)} lines; phis with an undef/poison input: {len(undef)}")
    for u in undef:
        print("   ", u[:160])
    # the flush: five wave reductions (update.dpp chains) of the loop-exit counters, in acc order
    roots = []
    for l in body:
        m = re.search(r"update\.dpp\.i32\(i32 0, i32 (%\d+), i32 273,", l)
        if m and not re.match(r"%\d+", "") and m.group(1) in defs and defs[m.group(1)].startswith("phi"):
            roots.append(m.group(1))
    roots = roots[-5:]  # (the flush is the last five wave reductions, at the loop exit)
    print("flushed counters (acc[0..4]):", roots)
    for k, r in enumerate(roots):
        seen, stack, bad = set(), [r], []
        while stack:
            v = stack.pop()
            if v in seen or v not in defs:
                continue
            seen.add(v)
            d = defs[v]
            if ("undef" in d or "poison" in d) and (d.startswith("phi") or d.startswith("add") or d.startswith("select")):
                bad.append(f"{v} = {d[:120]}")
            if d.split()[0] in ("phi", "add", "sub", "select", "zext"):
                stack.extend(re.findall(r"%\d+", d))
        print(f"  acc[{k}] {r}: {len(seen)} values in its def-use chain, undef/poison among them: {bad or 'none'}")


def isa_checks(path):
    L = open(path).read().split("\n")
    st = [i for i, l in enumerate(L) if l.startswith(NAME + ":")][0]
    en = [i for i in range(st, len(L)) if L[i].startswith(".Lfunc_end")][0]
    K = L[st:en]
    meta = open(path).read()
    blk = meta[meta.find(".name:           " + NAME) - 2500:meta.find(".name:           " + NAME)]
    for key in ("private_segment_fixed_size", "sgpr_spill_count", "vgpr_count", "vgpr_spill_count"):
        m = re.findall(r"\." + key + r":\s+(\d+)", blk)
        print(f"ISA {key}: {m[-1] if m else '?'}")
    # flush atomics and the latch reloads
    for i, l in enumerate(K):
        if "global_atomic_add_x2" in l or "Folded Reload" in l and "offset:1" in l and "v2" in l:
            pass
    lat = [i for i, l in enumerate(K) if "%Flow1058" in l]
    if lat:
        print("bucket-loop latch (reload + per-bucket increment):")
        for l in K[lat[0]:lat[0] + 24]:
            if "Reload" in l or "v_add_u32_e32 v2" in l or "v_add_u32_e32 v19" in l:
                print("   ", l.strip())


if __name__ == "__main__":
    isa_checks(sys.argv[1])
    ir_checks(sys.argv[2])
