"""CPU oracle for CatEars' fbank -> CMVN -> nnet path.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
package, and only as the checker / CPU baseline -- never as the product path.
"""
