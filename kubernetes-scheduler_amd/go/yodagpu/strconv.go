package yodagpu

import "strconv"

// The reference calls strconv directly; these wrappers keep its exact call shapes.

// sort.GetPodPriority (sort.go:12-18): `pri, _ := strconv.Atoi(p)`.
func strconvAtoi(s string) (int, error) { return strconv.Atoi(s) }

// algorithm.go:103: `Rio, _ := strconv.ParseFloat(pod.Annotations["diskIO"], 32)`.
func strconvParseFloat32(s string) (float64, error) { return strconv.ParseFloat(s, 32) }
