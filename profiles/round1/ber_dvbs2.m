EbN0=[-2 -1 0 1 2 3 ];
figure(1);
ber0=[0.2134 0.1864 0.1588 0.1312 0.1039 0.07872 ];
plot(EbN0, ber0, 'or--');
hold;
ber1=[0.2134 0.1864 0.1588 0.1312 0.1039 0.07872 ];
plot(EbN0, ber1, 'og-');
ber2=[0.2459 0.2195 0.1886 0.1352 0.0315 0.001506 ];
plot(EbN0, ber2, 'ob-');
ber3=[0.2176 0.187 0.1541 0.1181 0.07919 0.04113 ];
plot(EbN0, ber3, 'om-');
grid on;
hold off;
title('Bit Error Rate');
legend('BPSK', 'BitFlip', 'LogDomainSimple', 'SumProduct');
xlabel('EbN0');
ylabel('BER');
figure(2);
fer0=[
64, 64, 64, 64, 64, 64
];
plot(EbN0, fer0, 'or:');
hold;
fer1=[
64, 64, 64, 64, 64, 64
];
plot(EbN0, fer1, 'og-');
fer2=[
64, 64, 64, 64, 64, 64
];
plot(EbN0, fer2, 'ob-');
fer3=[
64, 64, 64, 64, 64, 64
];
plot(EbN0, fer3, 'om-');
grid on;
hold off;
title('Frame Errors');
legend('BPSK', 'BitFlip', 'LogDomainSimple', 'SumProduct');
xlabel('EbN0');
ylabel('FER');
