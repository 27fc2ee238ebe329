# connected components of an R-MAT graph + component-size histogram (OINK script)
# run: oink -in in.cc [-var scale 16]
variable scale index 16
variable t equal time
variable p equal nprocs

rmat ${scale} 2 0.25 0.25 0.25 0.25 0.0 12345 -o NULL mre
edge_upper -i mre -o NULL mre
cc_find 0 -i mre -o tmp.cc mrc
print "CC: $t secs on $p procs"
cc_stats -i mrc
