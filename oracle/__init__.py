"""ORACLE — test infrastructure only. NOT part of the product path.

CPU restatement of the reference's hot path (samuelstevens/hierarchical-vision
@ /root/reference), written from scratch to check the HIP path:

* ``index_ref``     numpy, integer/byte work: relative-position index, log-spaced
                    coords table, shift masks, shift+partition gather maps
                    (swinv2.py:69-102, 147-190, 328-388, 399-429) -- bit-exact.
* ``hierarchy_ref`` pure Python: taxonomy-path assignment (hierarchy.py:202-286,
                    429-485) -- bit-exact; multitask CE (hierarchy.py:65-94);
                    HXE (not implemented by the reference, hierarchy.py:183-185:
                    PARITY UNPINNED, pinned only by closed-form known answers).
* ``swinv2_ref``    torch CPU fp32 functional restatement of swinv2.py's
                    SwinTransformerV2 forward (swinv2.py:43-845).

Pinning: every function here is checked against golden vectors produced by
importing the reference itself in the build container
(``tests/golden/make_golden.py`` -> ``tests/golden/*.npz``; see
``tests/test_oracle_golden.py``).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this package, and only as the checker or as
the timed CPU baseline -- never as the thing measured or shipped.  The product
package (``hierarchical-vision_amd/``) never imports it.
"""
