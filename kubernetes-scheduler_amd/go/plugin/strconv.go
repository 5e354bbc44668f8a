package yoda

import "strconv"

func strconvAtoi(s string) (int, error) { return strconv.Atoi(s) }
