"""CPU oracle -- TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(),
bench.py's cpu_baseline leg).  Never imported by the product package."""
