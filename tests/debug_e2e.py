import sys, os
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, refharness as R, koboldcpp_amd.lib as K
g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'e2e_tiny.npz'))
R.lib().orc_set_fa_f32_accum(1)
hp = dict(R.TINY)
E = hp['n_embd']
for tag, types in (('q4km', R.q4_k_m_types(2)), ('q8_0', R.uniform_types(2, R.Q8_0))):
    full = g['q4km_prompt']
    for T in (16, 17, 37):
        prompt = full[:T]
        m = K.Model(hp, types); m.synth(1234)
        a = m.decode(prompt, 0); hid = m.read_hidden(T * E).reshape(T, E); m.close()
        o = R.OracleLlama(hp, types, 1234); lo = o.eval(prompt, 0)
        oh = np.empty(E, np.float32); R.lib().orc_llama_last_hidden(o.m, R.ptr(oh))
        d = np.abs(a - lo); dh = np.abs(hid[-1] - oh)
        print(os.environ.get('KCPP_FA_PATH', '0'), tag, T, 'logits median %.2e max %.2e | last hidden median %.2e max %.2e' % (np.median(d), d.max(), np.median(dh), dh.max()), flush=True)
