"""Shared work-request cases for the segmentation tests (CPU and GPU)."""
from __future__ import annotations

import numpy as np

import segment_oracle as SO
from roce_icrc import engine as E

SRC_IP = 0x0A010130  # 10.1.1.48
DST_IP = 0x0A01010F  # 10.1.1.15


def to_records(wrs: list[SO.SegWR]) -> np.ndarray:
    rec = E.seg_wrs(len(wrs))
    for i, w in enumerate(wrs):
        rec[i]["op"] = w.op
        rec[i]["mr_offset"] = w.mr_offset
        rec[i]["length"] = w.length
        rec[i]["psn"] = w.psn
        rec[i]["dqpn"] = w.dqpn
        rec[i]["src_ip"] = w.src_ip
        rec[i]["dst_ip"] = w.dst_ip
        rec[i]["sport"] = w.sport
        rec[i]["flags"] = w.flags
        rec[i]["imm"] = w.imm
        rec[i]["remote_va"] = w.remote_va
        rec[i]["rkey"] = w.rkey
        rec[i]["msn"] = w.msn
        rec[i]["swap"] = w.swap
        rec[i]["comp"] = w.comp
    return rec


def lengths_for(pmtu: int) -> list[int]:
    """Message lengths around every boundary the rules have: empty, pad 1-3,
    exactly one PMTU, one byte over, several packets with a ragged tail."""
    return [0, 1, 2, 3, 4, 5, 17, pmtu - 1, pmtu, pmtu + 1, 2 * pmtu, 3 * pmtu + 2]


def all_ops_cases(pmtu: int, mr_size: int, seed: int = 0) -> list[SO.SegWR]:
    rng = np.random.default_rng(seed)
    wrs = []
    for op in range(SO.ATOMIC_ACK + 1):
        # header-only ops: lengths only reach RETH.dlen (READ_REQUEST)
        for length in lengths_for(pmtu) if op < SO.READ_REQUEST else (0, 5, 3 * pmtu + 2):
            for flags in (0, SO.SIGNALED | SO.SOLICITED):
                off = int(rng.integers(0, mr_size - length + 1))
                wrs.append(SO.SegWR(
                    op=op, mr_offset=off, length=length,
                    psn=int(rng.integers(0, 1 << 24)), dqpn=int(rng.integers(0, 1 << 24)),
                    src_ip=SRC_IP, dst_ip=DST_IP, sport=int(rng.integers(0, 1 << 16)),
                    flags=flags, imm=int(rng.integers(0, 1 << 32)),
                    remote_va=int(rng.integers(0, 1 << 63)), rkey=int(rng.integers(0, 1 << 32)),
                    msn=int(rng.integers(0, 1 << 24)),
                    swap=int(rng.integers(0, 1 << 63)) * 2 + 1, comp=int(rng.integers(0, 1 << 63))))
    return wrs
