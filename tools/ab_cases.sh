# The layouts the round-4 bench lines run (autotune's picks), for tools/variant_check.py --cases
C2=2:4096:4:16:1:1:0:1:1
C3=3:65536:4:16:4:4:1:2:0
C4=4:32768:4:16:1:4:2:2:0
C5=5:16384:8:8:1:4:2:2:0
ALL=$C2,$C3,$C4,$C5
