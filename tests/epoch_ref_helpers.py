"""Shared oracle helper for the epoch tests: one instance's expected results."""
from oracle import epoch_np as onp


def oracle_epoch(inst, b):
    """(new balance, applied, next-cycle balance, vote, total, winner) of instance ``b``
    (blockchain/core.go:433-464 via the numpy oracle)."""
    bal = inst["balance"][b]
    s, e = inst["start"][b], inst["end"][b]
    natt = inst["natt"]
    bo = inst["boffs"][b * natt:(b + 1) * natt + 1]
    v, t = onp.crosslink_tallies(inst["committee"], inst["coffs"], inst["att_comm"][b * natt:(b + 1) * natt],
                                 inst["bits"], bo, bal)
    win = onp.crosslink_winners(v, t, inst["att_shard"][b * natt:(b + 1) * natt], inst["rec_dynasty"][b],
                                int(inst["dynasty"][b]))
    nb, applied = onp.calculate_rewards(bal, s, e, int(inst["dynasty"][b]), int(inst["total_deposit"][b]),
                                        inst["bits"], bo)
    return nb, applied, onp.active_balance_sum(nb, s, e, int(inst["dynasty"][b])), v, t, win
