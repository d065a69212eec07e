bash tools/r04_s3.sh r04c && bash tools/r04_s4.sh r04d
