"""ICRC error hooks for the reference's hooks framework.

datenlord/roce-sim corrupts packets from Python hook functions
(src/hooks.py:10-138) registered per QP by SideServicer.SetHook
(src/sanity_side.py:345-364) as one of three types: a SEND hook
``(wr_ssn, req_pkt, real_send) -> same`` called before the requester builds
a packet (src/roce_sq.py:1205-1214), a RESP hook ``(resp_pkt, save_resp_pkt)
-> same`` on the responder (src/roce_rq.py:714-716), and a RECV hook
``(pkt) -> pkt`` on receive.  Its hooks edit BTH / RETH / AETH fields or the
payload; none can produce an ICRC error, because the ICRC is computed after
the hook and never checked.  The hooks below add that case: the packet is
built with its true ICRC XOR a non-zero mask (``BTH.icrc_fault``), so it goes
out with a wrong ICRC and a consistent UDP checksum, and the engine's verify
path (``verify_frames`` / ``recv_datagrams``) must drop it.  For whole batches
already in HBM, ``IcrcEngine.inject_faults_dev`` does the same on the GPU.
"""
from __future__ import annotations

from enum import IntEnum
from typing import Callable, Iterable, Optional

from .roce import BTH


class HOOK_TYPE(IntEnum):  # src/hooks.py:10-13
    SEND = 0
    RECV = 1
    RESP = 2


def _mark(pkt, psns: Optional[set], mask: int):
    bth = pkt.getlayer(BTH)
    if bth is not None and (psns is None or bth.psn in psns):
        bth.__dict__["icrc_fault"] = mask
    return pkt


def icrc_error_send_hook(wr_ssn, req_pkt, real_send):
    """SEND hook: every request packet leaves with a wrong ICRC."""
    return wr_ssn, _mark(req_pkt, None, 1), real_send


def icrc_error_resp_hook(resp_pkt, save_resp_pkt):
    """RESP hook: every response packet leaves with a wrong ICRC."""
    return _mark(resp_pkt, None, 1), save_resp_pkt


def make_icrc_error_send_hook(psns: Iterable[int], mask: int = 1) -> Callable:
    """A SEND hook corrupting the ICRC of the packets with these PSNs only
    (the PSN-selective style of src/hooks.py, e.g. sim_read_partial_retry_hook)."""
    if mask & 0xFFFFFFFF == 0:
        raise ValueError("mask must be non-zero")
    sel = set(psns)
    return lambda wr_ssn, req_pkt, real_send: (wr_ssn, _mark(req_pkt, sel, mask), real_send)


def make_icrc_error_resp_hook(psns: Iterable[int], mask: int = 1) -> Callable:
    """A RESP hook corrupting the ICRC of the responses with these PSNs only."""
    if mask & 0xFFFFFFFF == 0:
        raise ValueError("mask must be non-zero")
    sel = set(psns)
    return lambda resp_pkt, save_resp_pkt: (_mark(resp_pkt, sel, mask), save_resp_pkt)
