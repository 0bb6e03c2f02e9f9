import sys
for line in open(sys.argv[1]):
    t, rest = line.split('|',1)
    ks = rest.split()
    cats = {}
    for k in ks:
        name, _, cnt = k.rpartition('x')
        base, _, stream = name.partition('@')
        c = 'PR' if base in ('tr_a','fx_b','weights_batch','tr_cut_b','kind_insert_b','kind_verify_b','pref_apply_b','pref_partial_b','pref_total_b','reset_init_b') else ('SP' if base=='win_spectrum' else 'B')
        cats[c] = cats.get(c,0) + int(cnt)
    print(t.split('busy')[0].strip(), t.split('busy-sum')[1].strip(), ' '.join(f"{k}:{v}" for k,v in sorted(cats.items())))
