"""ICRC error hooks (roce_icrc.hooks) without a GPU: the hook signatures and
PSN selection of src/hooks.py, and the BTH.icrc_fault mark they set."""
import pytest

from roce_icrc import hooks as H
from roce_icrc import roce as R


def test_hook_types_match_reference():
    assert (H.HOOK_TYPE.SEND, H.HOOK_TYPE.RECV, H.HOOK_TYPE.RESP) == (0, 1, 2)  # src/hooks.py:10-13


def test_send_hook_marks_selected_psns_only():
    hook = H.make_icrc_error_send_hook([3, 5], mask=0x80)
    for psn in range(8):
        pkt = R.BTH(opcode=0x04, psn=psn, dqpn=1) / R.Raw(load=b"abcd")
        ssn, out, real = hook(7, pkt, True)
        assert ssn == 7 and real is True
        assert out[R.BTH].icrc_fault == (0x80 if psn in (3, 5) else 0)


def test_resp_hook_and_copy_keep_the_mark():
    pkt = R.BTH(opcode=0x10, psn=1) / R.AETH(code=0, value=31, msn=2)
    out, save = H.icrc_error_resp_hook(pkt, True)
    assert save is True and out[R.BTH].icrc_fault == 1
    assert out.copy()[R.BTH].icrc_fault == 1


def test_zero_mask_rejected():
    with pytest.raises(ValueError):
        H.make_icrc_error_resp_hook([1], mask=0)
