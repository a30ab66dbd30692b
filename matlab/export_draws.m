function export_draws(Y, g, k, BURNIN, MCMC, thin, rho, s, fname)
% EXPORT_DRAWS  MATLAB-side exporter for true MATLAB parity (SURVEY §8(c), §8(f) row 1).
%
% Replays, from rng(s), the standard variates that divideconquer.m consumes from MATLAB's
% global stream (SURVEY Appendix B: same calls, same order, standard parameters — gamrnd(a,b)
% draws b.*randg(a) and normrnd(0,1,sz) draws randn(sz)), then resets rng(s) and runs the
% user's own divideconquer(Y,g,k,BURNIN,MCMC,thin,rho) on the same stream, and saves both:
% the draws in the layout libdcfm's injected-draws mode reads (include/dcfm.h,
% dcfm_draws_view) and the reference's Sigmaout.  tests/test_matlab_parity.py consumes the
% file (DCFM_MATLAB_DRAWS=<fname>): oracle and GPU chains driven by these draws must
% reproduce this Sigmaout to 1e-10.  Needs MATLAB + Statistics Toolbox; not runnable in
% the build container (no MATLAB there).
%
% Hyper-parameters are the reference's fixed values (dc:62-65): as=1, bs=0.3, df=3,
% ad1=2, bd1=1, ad2=2, bd2=1.

as = 1; df = 3; ad1 = 2; ad2 = 2;
n = size(Y, 1);
nz = arrayfun(@(j) nnz(Y(:, j)), 1:size(Y, 2));       % dc:31-34 (draws nothing)
p = sum(nz > 0);
P = p / g; K = k / g; N = BURNIN + MCMC;
assert(P == fix(P) && K == fix(K), 'P = p/g and K = k/g must be integers (dc:41)');

rng(s);
% ---- init, dc:50-83 --------------------------------------------------------------
varind = randperm(p);                                  % dc:50
ps0 = randg(as, [P, 1, g]);                            % dc:69   (scaled by 1/bs there)
X0 = randn(n, K);                                      % dc:71
psi0 = randg(df / 2, [P, K, g]);                       % dc:73   (scaled by 2/df)
Z0 = zeros(n, K, g); delta0 = zeros(K, g);
for m = 1:g                                            % dc:79-87
    Z0(:, :, m) = randn(n, K);
    delta0(1, m) = randg(ad1);
    if K > 1
        delta0(2:K, m) = randg(ad2, [K - 1, 1]);
    end
end
% ---- per iteration, dc:90-177, in consumption order -------------------------------
NZ = zeros(K, n, g, N); NX = zeros(K, n, N); NL = zeros(K, P, g, N);
Gpsi = zeros(P, K, g, N); Gdelta = zeros(K, g, N); Gps = zeros(P, g, N);
for t = 1:N
    for m = 1:g, for i = 1:n, NZ(:, i, m, t) = randn(K, 1); end, end          % dc:104
    for i = 1:n, NX(:, i, t) = randn(K, 1); end                                % dc:126
    for m = 1:g, for j = 1:P, NL(:, j, m, t) = randn(K, 1); end, end          % dc:142
    for m = 1:g, Gpsi(:, :, m, t) = randg(df / 2 + 0.5, [P, K]); end          % dc:150
    for m = 1:g                                                                % dc:158,163
        Gdelta(1, m, t) = randg(ad1 + 0.5 * P * K);
        for h = 2:K, Gdelta(h, m, t) = randg(ad2 + 0.5 * P * (K - h + 1)); end
    end
    for m = 1:g, Gps(:, m, t) = randg(as + 0.5 * n, [1, P])'; end             % dc:170
end
% ---- the reference itself on the same stream ---------------------------------------
rng(s);
Sigmaout = divideconquer(Y, g, k, BURNIN, MCMC, thin, rho);
save(fname, 'Y', 'g', 'k', 'BURNIN', 'MCMC', 'thin', 'rho', 'varind', 'ps0', 'X0', 'psi0', ...
     'Z0', 'delta0', 'NZ', 'NX', 'NL', 'Gpsi', 'Gdelta', 'Gps', 'Sigmaout', '-v7');
end
