"""CPU oracle for the MI355X DPEngine.aggregate hot path.

TEST INFRASTRUCTURE.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import, call, link or execute anything under oracle/,
and only as the checker (or the timed CPU baseline) -- never as the product
path.  Parity pinning: see oracle/dp_oracle.c and DESIGN.md section
"Oracle".
"""
