"""Report text: the NS_LOG_INFO lines of PrintStatistics (p2pnetwork.cc:255-284) and
PrintPeriodicStats (:233-249), uint32 accumulators included."""
import numpy as np


def _stats(gossip, **kw):
    n = 2
    base = dict(gen=[3, 4], recv=[10, 9], fwd=[10, 9], sent=[26, 13], processed=[13, 13],
                peers=[2, 1], sockets=[1, 1])
    base.update(kw)
    return gossip.Stats(**{k: np.asarray(v, np.uint64 if k == "sent" else np.uint32)
                           for k, v in base.items()})


def test_statistics_text(gossip):
    txt = gossip.format_statistics(_stats(gossip))
    assert txt == (
        "=== P2P Gossip Network Simulation Statistics ===\n"
        "Node 0: Generated 3, Received 10, Forwarded 10, Total sent 26, Total processed 13, "
        "Peer count 2, Socket connections 1\n"
        "Node 1: Generated 4, Received 9, Forwarded 9, Total sent 13, Total processed 13, "
        "Peer count 1, Socket connections 1\n"
        "Total shares generated: 7\n"
        "Total shares received: 19\n"
        "Total shares forwarded: 19\n"
        "Total shares sent: 39\n"
        "Total socket connections: 2\n")


def test_statistics_uint32_wrap(gossip):
    # sharesSent is uint32_t (p2pnode.h:40) and the totals are uint32_t (:257-261).
    st = _stats(gossip, sent=[2**32 + 5, 2**32 - 1])
    txt = gossip.format_statistics(st)
    assert "Total sent 5," in txt and "Total sent 4294967295," in txt
    assert "Total shares sent: 4\n" in txt


def test_periodic_text(gossip):
    txt = gossip.format_periodic(10.0, 10, 14, 140, 26)
    assert txt == ("=== Periodic Stats at 10s ===\n"
                   "Total shares generated: 14\n"
                   "Average shares per node: 14\n"
                   "Total socket connections: 26\n")
    # integer division of the uint32 total (p2pnetwork.cc:248)
    assert "Average shares per node: 3\n" in gossip.format_periodic(20.0, 7, 1, 27, 0)
