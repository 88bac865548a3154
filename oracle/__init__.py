"""CPU oracle for the WSWGAT hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may
import this package, and only as the checker / the timed CPU baseline.  The
product package (hetersumgraph_amd) never imports it.

* ``oracle.fused``   -- float64 edge-wise restatement (parity checker), pinned
                        to the golden vectors in tests/golden/.
* ``oracle.masks``   -- numpy restatement of the kernels' dropout-mask
                        generators (head-projection keep-bits, FFN hash), so
                        the train-mode stack is checked with the same masks.
* ``oracle.dgl_udf`` -- float32 restatement structured like DGL 0.4's UDF
                        execution (per head apply_edges + degree-bucketed pull),
                        the "DGL-CPU" baseline timed by bench.py (kind "port").
"""
