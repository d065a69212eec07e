bash tools/r04_s2.sh r04e && bash tools/r04_s4.sh r04f
