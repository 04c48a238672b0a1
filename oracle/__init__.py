"""ORACLE package — test infrastructure only.

CPU restatements of the reference's SFNO-Block path used as the parity checker
(tests/, __graft_entry__.smoke) and as bench.py's cpu_baseline leg.  The product
package (modulated-spherical-fourier-neural-operator_amd/msfno_amd) never
imports anything from here.
"""
