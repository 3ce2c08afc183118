"""CPU oracle for the TransMVSNet depth-inference hot path -- TEST INFRASTRUCTURE ONLY.

Importable only from ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg, where it is the checker (or the timed CPU baseline), never the
thing measured or shipped. ``transmvsnet_amd`` must not import it.

Pinned against golden vectors captured from the real reference
(``tests/golden/make_golden.py``; see DESIGN.md "Oracle").
"""
